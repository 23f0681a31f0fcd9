"""Experiment-only (after apply_stamps.py): a workgroup-level end stamp (9) on the
non-fused k_step path (headline), behind one extra barrier."""
import sys
R = sys.argv[1]
p = R + "mrts_engine.hip"
s = open(p).read()
a = "    emit_outputs<NT, P, OT>(p, L, G, true, p.mask != nullptr, botg ? 64 : 0);\n"
assert a in s
s = s.replace(a, a + """    if (!FB) {
        __syncthreads();
        if (threadIdx.x == 0) stamp(blockIdx.x, 9);
    }
""")
a2 = """    if (threadIdx.x < 6 * G.nviews) {
        int v = threadIdx.x / 6, k = threadIdx.x % 6;"""
assert a2 in s
open(p, "w").write(s)
print("head stamps")
