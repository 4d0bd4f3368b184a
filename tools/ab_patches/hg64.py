"""A/B patch: the two-in-flight half grid for passes up to 64 GiB (0: never)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "api.cpp")
    s = open(p).read()
    old = "constexpr uint64_t kHalfGridMaxBytes = 16ull << 30;"
    assert old in s
    open(p, "w").write(s.replace(old, "constexpr uint64_t kHalfGridMaxBytes = 64ull << 30;"))
