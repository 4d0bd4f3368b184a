"""A/B patch: K10 (marshal mode) launched for 7 waves/SIMD instead of 8 (more VGPRs, fewer spills)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "tokenize.hip")
    s = open(p).read()
    old = "k_encode_docs<8, kModeMarshal><<<"
    assert old in s
    open(p, "w").write(s.replace(old, "k_encode_docs<7, kModeMarshal><<<"))
