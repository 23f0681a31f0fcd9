"""Experiment-only: instrument the fused k_step / bot_game with wall_clock64 stamps."""
import sys
R = sys.argv[1] if len(sys.argv) > 1 else "/root/repo/microrts-py_amd/csrc/"
def sub(path, a, b, count=1):
    s = open(R + path).read()
    assert a in s, (path, a[:60])
    s = s.replace(a, b, count)
    open(R + path, "w").write(s)
sub("mrts_engine.h", "struct EngineParams {", """#define MRTS_STAMPS 12
static __device__ unsigned long long g_stamps[8192 * MRTS_STAMPS];
__device__ __forceinline__ void stamp(int g, int k) { g_stamps[(size_t)g * MRTS_STAMPS + k] = wall_clock64(); }
struct EngineParams {""")
sub("mrts_engine.hip", """    __builtin_amdgcn_s_setprio(2);""", """    __builtin_amdgcn_s_setprio(2);
    if (threadIdx.x == 0) stamp(blockIdx.x, 0);""")
sub("mrts_engine.hip", """        L.aux[c] = nw;
    }
    __syncthreads();""", """        L.aux[c] = nw;
    }
    __syncthreads();
    if (threadIdx.x == 0) stamp(blockIdx.x, 11);""")
sub("mrts_engine.hip", """    __syncthreads();
    // (4) GameState.cycle(): time++, execute ready assignments in issue order""", """    __syncthreads();
    if (threadIdx.x == 0) stamp(blockIdx.x, 1);
    // (4) GameState.cycle(): time++, execute ready assignments in issue order""")
sub("mrts_engine.hip", """    // (7) write back + one-hot observation of every view
    store_game<NT>(p, L, g);""", """    // (7) write back + one-hot observation of every view
    if (threadIdx.x == 0) stamp(blockIdx.x, 2);
    store_game<NT>(p, L, g);""")
sub("mrts_engine.hip", """        else
            emit_outputs<NT, P, OT>(p, L, G, true, p.mask != nullptr, 64, early_cnt);
        return;""", """        else
            emit_outputs<NT, P, OT>(p, L, G, true, p.mask != nullptr, 64, early_cnt);
        if (threadIdx.x == 64) stamp(blockIdx.x, 7);
        return;""")
sub("mrts_engine.hip", """extern "C" {
hipError_t mrts_engine_reset(""", """extern "C" {
int mrts_debug_stamps(unsigned long long* out, int n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * MRTS_STAMPS * n, 0, hipMemcpyDeviceToHost);
}
hipError_t mrts_engine_reset(""")
sub("mrts_bots.h", """    const int map = gs[MRTS_G_MAP];""", """    const int map = gs[MRTS_G_MAP];
    if (FUSED && lane0()) stamp(blockIdx.x, 3);""")
sub("mrts_bots.h", """    // units in pgs.units order: ordered compaction by cell, then rank by uid""", """    if (FUSED && lane0()) stamp(blockIdx.x, 8);
    // units in pgs.units order: ordered compaction by cell, then rank by uid""")
sub("mrts_bots.h", """    S.rurow = 0;
    {""", """    if (FUSED && lane0()) stamp(blockIdx.x, 9);
    S.rurow = 0;
    {""")
sub("mrts_bots.h", """    const bool table = S.ai != MRTS_AI_RANDOM_BIASED && S.ai != MRTS_AI_RANDOM;""", """    if (FUSED && lane0()) stamp(blockIdx.x, 10);
    const bool table = S.ai != MRTS_AI_RANDOM_BIASED && S.ai != MRTS_AI_RANDOM;""")
sub("mrts_bots.h", """    switch (S.ai) {
    case MRTS_AI_WORKER_RUSH""", """    if (FUSED && lane0()) stamp(blockIdx.x, 4);
    switch (S.ai) {
    case MRTS_AI_WORKER_RUSH""")
sub("mrts_bots.h", """        behaviours_parallel(S, L, 0, false, true);
        translate_actions(S, L);""", """        behaviours_parallel(S, L, 0, false, true);
        if (lane0()) stamp(blockIdx.x, 5);
        translate_actions(S, L);""")
sub("mrts_bots.h", """    for (int i = lane; i < S.npa; i += BT) pa_g[i] = L.pa[i];""", """    if (FUSED && lane0()) stamp(blockIdx.x, 6);
    for (int i = lane; i < S.npa; i += BT) pa_g[i] = L.pa[i];""")
print("stamped")
