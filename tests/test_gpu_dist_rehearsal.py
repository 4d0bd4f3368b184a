"""The N > 1 bench path executed on hardware: two ranks on the one leased MI355X.

RCCL refuses two ranks on one device, so `bench.py --dist-backend gloo` runs the real multi-rank path --
the self-launch child (torch.distributed.run), byte-weighted LPT shards with the weight all-reduce,
per-rank engines on GPU 0, the one all-gather per step, the max-dt and total-pairs all-reduces, rank 0's
relayed line -- with counts and IDs staged through host tensors.  Both collectives run: one pass in flight
(DirtyGather, export copies into the host tensors) and the default two passes in flight (PipelinedGather:
two contexts, a view of the resident batch, the engine-written send buffer of each pass staged to the host
after it, lookahead count checks), the latter also with capacities forced below the counts so the lookahead
regrow re-gathers steps s and s + 1 at world 2.  The node-wide dirty sets rank 0 gathered must equal a
single-rank diff of the whole population."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("pipeline,cap_frac", [(1, 1.0), (2, 1.0), (2, 0.5)])
def test_bench_two_ranks_gloo_on_one_gpu(tmp_path, pipeline, cap_frac):
    dump = str(tmp_path / "gather.npz")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--pairs", "100000", "--clusters", "1000",
           "--dist-backend", "gloo", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--sample", "0",
           "--json-in-pairs", "0", "--threads", "8", "--dump-gather", dump, "--pipeline", str(pipeline),
           "--gather-cap-frac", str(cap_frac), "--calib-passes", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["shard"]["rule"] == "LPT by sum of B_pair"
    assert line["config"]["passes_in_flight"] == pipeline
    g = line["checks"]["gather"]
    assert g["pipeline"] == pipeline and g["engine_writes_send_buffer"] == (pipeline == 2)
    assert g["regrows"] == (1 if cap_frac < 1 else 0), g
    assert g["capacity_ok"] and g["node_sets_eq_truth"], json.dumps(line["checks"]) + r.stderr[-2000:]
    assert g["gathered_spec"] == g["node_spec_dirty"] == g["node_expected_spec"]
    assert g["gathered_status"] == g["node_status_dirty"] == g["node_expected_status"]
    assert line["checks"]["full_size"]["flag_mismatches"] == 0
    got = np.load(dump)
    # one rank, the whole population, on the same GPU
    cfg = S.make_cfg("config3", n_pairs=100000, n_clusters=1000)
    pop = S.Population(cfg)
    e = G.Engine(device=0, encode_threads=8)
    ch = pop.chunk(e, 0, pop.n, 8)
    db = e.device_batch(ch.pool_bytes + 4096, pop.n)
    db.append(ch.hb)
    res = e.wait(e.diff(db))
    assert np.array_equal(np.sort(got["spec"].astype(np.uint32)), np.sort(res.spec_dirty_ids))
    assert np.array_equal(np.sort(got["status"].astype(np.uint32)), np.sort(res.status_dirty_ids))
    assert got["spec"].size > 100 and got["status"].size > 1000
    db.free()
    ch.hb.free()
    e.close()
