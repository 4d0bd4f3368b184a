"""A/B patch: >= 12 items per resident wave before 64-pair chunks stop splitting (config2 / the N = 8 share: 16-pair
items instead of 32)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "constexpr uint32_t kK2ItemsPerWave = 6;"
    assert old in s
    open(p, "w").write(s.replace(old, "constexpr uint32_t kK2ItemsPerWave = 12;"))
