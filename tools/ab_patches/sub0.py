"""A/B patch: >= 4 items per resident wave before 64-pair chunks are split (config2: whole 64-pair items)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "constexpr uint32_t kK2ItemsPerWave = 6;"
    assert old in s
    open(p, "w").write(s.replace(old, "constexpr uint32_t kK2ItemsPerWave = 4;"))
