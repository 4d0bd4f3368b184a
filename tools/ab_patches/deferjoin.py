"""A/B patch: K2 joins no dirty pair itself -- every join that fits a whole deferral (<= 1024 merged keys) goes to
K3's compaction waves (join_whole, staged in LDS), larger ones to K4's slices; K2 only streams and writes
sentinel-only pairs' paths."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = "            if (used + ck <= arena_per_wave && ck <= (tail_round ? kTailJoinMax : kDeepJoin)) {"
    assert old in s
    s = s.replace(old, "            if (!(fk & (F_JSPEC | F_JSTAT)) && used + ck <= arena_per_wave && "
                       "ck <= (tail_round ? kTailJoinMax : kDeepJoin)) {")
    open(p, "w").write(s)
