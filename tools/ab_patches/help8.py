"""A/B patch: the default (8 chunks a side) kernel with the block-cooperative final round (HELP: idle waves stream
passes of their siblings' items) -- 128 VGPRs, still 4 waves/SIMD."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "default: return k_compare_flat<8, 1>;"
    assert old in s
    open(p, "w").write(s.replace(old, "default: return k_compare_flat<8, 1, false, true>;"))
