"""A/B patch: K2's grid held to 2 resident blocks per CU (2 waves/SIMD) whatever the kernel's occupancy."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "    return 256u * (uint32_t)occ[v];\n}"
    assert old in s
    open(p, "w").write(s.replace(old, "    return 256u * (uint32_t)std::min(occ[v], 2);\n}"))
