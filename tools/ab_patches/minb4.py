"""A/B patch: the default K2 kernel held to 4 waves/SIMD (128 VGPRs; the compiler spills what does not fit)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "default: return k_compare_flat<8, 1>;"
    assert old in s
    open(p, "w").write(s.replace(old, "default: return k_compare_flat<8, 4>;"))
