"""Debug: HIP runtimes mapped into a process that uses torch.distributed (RCCL) and libgpudiff."""
import socket
import sys

sys.path.insert(0, ".")
from kcp_amd import gpudiff as G  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def maps():
    with open("/proc/self/maps") as f:
        return sorted({l.split()[-1] for l in f if "amdhip" in l or "hsa-runtime" in l})


print("before torch cuda:", G.device_count(), maps(), flush=True)
torch.cuda.set_device(0)
print("after set_device:", G.device_count(), torch.cuda.device_count(), flush=True)
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
print("after init_process_group:", G.device_count(), maps(), flush=True)
t = torch.ones(4, device="cuda")
dist.all_reduce(t)
print("after all_reduce:", G.device_count(), t.tolist(), flush=True)
e = G.Engine(device=0)
print("engine ok", flush=True)
e.close()
dist.destroy_process_group()
