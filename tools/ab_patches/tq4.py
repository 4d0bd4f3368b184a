"""A/B patch: the launch's tail of half-size items twice as long (kK2TailQuarters 2 -> 4)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.h")
    s = open(p).read()
    old = "constexpr uint32_t kK2TailQuarters = 2;"
    assert old in s
    open(p, "w").write(s.replace(old, "constexpr uint32_t kK2TailQuarters = 4;"))
