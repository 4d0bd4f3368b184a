"""A/B patch: K2 joins small pairs from global memory again (no LDS staging in K2; K3's whole deferrals keep it)."""
import os


def patch(root):
    p = os.path.join(root, "kcp_amd", "csrc", "kernels.hip")
    s = open(p).read()
    old = """                    if (sa <= kJoinLdsSide && sb <= kJoinLdsSide) {  // small pair: joined from LDS
                        stage_pair(my_lds, pool, r.off_a, sa, r.off_b, sb, lane);"""
    assert old in s
    s = s.replace(old, """                    if (false && sa <= kJoinLdsSide && sb <= kJoinLdsSide) {  // small pair: joined from LDS
                        stage_pair(my_lds, pool, r.off_a, sa, r.off_b, sb, lane);""")
    old = "    __shared__ __attribute__((aligned(16))) uint8_t join_lds[4][2 * kJoinLdsSide];  // stage_pair, one area per wave\n    uint8_t* const my_lds = join_lds[threadIdx.x >> 6];\n    [[maybe_unused]] HelpSlot"
    if old not in s:
        old = None
    open(p, "w").write(s)
