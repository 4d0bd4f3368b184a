import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import bench_upsert
from kcp_amd import gpudiff as G
from kcp_amd import synth as S
n = 131072
pop = S.Population(S.make_cfg("config3"))
buf, offs, _ = pop.json_range(0, n, 16)
docs = [bench_upsert.add_owner_refs(bytes(buf[offs[2 * i + 1]:offs[2 * i + 2]]), i) for i in range(n)]
eng = G.Engine(device=0)
res = eng.upsert_bodies(docs)
bad = 0
os.makedirs("gpurun_out/dbg", exist_ok=True)
for i in range(n):
    h = G.upsert_body_host(docs[i])
    if res.bodies[i] != h:
        bad += 1
        a, b = res.bodies[i], h
        k = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), min(len(a), len(b)))
        print(i, len(a), len(b), "dev:", a[max(0, k - 60):k + 40], "\nhost:", b[max(0, k - 60):k + 40])
        if bad <= 3:
            open("gpurun_out/dbg/doc%d.json" % i, "wb").write(docs[i])
print("bad", bad)
