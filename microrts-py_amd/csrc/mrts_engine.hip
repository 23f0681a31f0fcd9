// mrts_engine.hip -- gfx950 kernels of the vectorised MicroRTS engine.
//
// Restates, on the device, the Java path behind MicroRTSGridModeVecEnv
// (/root/reference/gym_microrts/envs/vec_env.py): JNIGridnetVecClient.reset
// (vec_env.py:279), .gameStep (vec_env.py:1002: JNIAI action decode, issueSafe
// p0/p1, GameState.cycle, the six ai.reward functions, auto-reset) and
// .getMasks (vec_env.py:1097), plus the python-side one-hot encoder
// _encode_obs (vec_env.py:311-321).  Rules: SURVEY.md Appendix A, DESIGN.md §4.
//
// Mapping: one workgroup per GAME, one lane per grid cell (16x16 -> 256 lanes),
// the game's cell records staged in LDS.  Everything that is per-cell runs
// lane-parallel (decode, legality, masks, readiness, one-hot); the parts of the
// Java that are inherently ordered (PlayerAction consistency filter, issue()
// conflict resolution, execution of ready actions in LinkedHashMap order) run
// on lane 0 over compact ballot-built lists, which hold only the few units
// that act this tick.  Outputs are written with 16-byte stores from compact
// per-cell bit words in LDS (one-hot obs: 1 word/cell, mask: 3 words/cell).
// A step launch takes a StepGroup: one or more engines (map-size buckets) cut
// into grid segments, bot games first (mrts_step_group).
//
// Integer work only: no MFMA, the kernels are HBM-bound on the obs/mask writes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "mrts_engine.h"
#include "mrts_layout.h"

#include "mrts_rules.h"
#include "mrts_bots.h"

namespace mrts {

// ---------------------------------------------------------------------------
// LDS carving (all dynamic, 16-byte aligned pieces: cdna_hip_programming §6 G17)
struct Lds {
    uint32_t* unit;
    int32_t* uid;
    uint32_t* act;
    uint32_t* seq;
    uint32_t* aux;   // decoded rows, then one-hot / mask bit words
    int32_t* resv;   // reservation holder per cell
    int32_t* list;   // compact cell lists
    int32_t* prod;   // pending produce cells
    int32_t* blist;  // the bot's PlayerAction order (bot games)
    int32_t* blist0; // player 0's bot PlayerAction (bot-vs-bot games)
    int4* snap;      // ready-action snapshots
    uint32_t* outw;  // emit_outputs one-hot words [NV][HW]: aliases resv .. snap (32 B per cell with outm)
    uint32_t* outm;  // emit_outputs mask words [NV][HW][3] (outw + 2 HW, unless the fused step places them)
    uint8_t* wall;
    unsigned long long* ballot;
    uint32_t* posbits;
    uint32_t* claim;   // [2][posw] target positions claimed by >= 1 / >= 2 rows this tick
    uint32_t* vis;   // [2][HW/32+1] cells observable by player 0 / 1 (partial obs)
    int* sc;         // scalars
};
// L.sc[0 .. MRTS_GENV_WORDS) mirrors genv (load_game / store_game)
enum { SC_TIME = MRTS_G_TIME, SC_RES0 = MRTS_G_RES0, SC_RES1 = MRTS_G_RES1, SC_UID = MRTS_G_NEXT_UID,
       SC_STEPS = MRTS_G_STEPS, SC_MAP = MRTS_G_MAP, SC_ERR = MRTS_G_ERR, SC_AA_N = MRTS_G_AA_N, SC_TICKS = MRTS_G_TICKS,
       SC_NPA = MRTS_G_NPA, SC_R0 = 16, /* rewards: [player][6] as ints */ SC_NPROD = 28, SC_RPROD = 29 /* ready produces */,
       SC_OVER = 30 /* a pending produce is over its owner's budget */,
       SC_HAS = 31 /* units of player 0 (bits 0..15) and player 1 (16..31) */,
       SC_PSUM = 32 /* [2] cost of the player's produce rows this tick */,
       SC_PMAX = 34 /* [2] largest cost among the player's pending produces */,
       SC_SERIAL = 36 /* the ready set executes in order */, SC_NPEND = 37 /* pending produces listed in L.prod */,
       SC_NREADY = 38 /* ready assignments listed in L.list */, SC_NLEFT = 39 /* rows (2a) left to the ordered path */,
       SC_WORDS = 40 };
static_assert(MRTS_GENV_WORDS <= SC_R0, "genv words overlap the LDS scalars");

typedef int v4i __attribute__((ext_vector_type(4)));

// 16-byte store of an output row segment (obs / masks: written once, read by
// the consumer after the kernel; plain stores measured 5 % faster than
// non-temporal ones)
__device__ __forceinline__ void st16(void* dst, int a, int b, int c, int d) {
    v4i v = {a, b, c, d};
    *reinterpret_cast<v4i*>(dst) = v;
}

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// L.vis: both players' visibility words (phase A), and before that the ballot
// words of the step's first compaction (one 8-B word per wave and NT cells)
__host__ __device__ inline size_t vis_bytes(int HW, int NT) {
    const size_t v = 8 * (size_t)(HW / 32 + 1), b = 8 * (size_t)((HW + NT - 1) / NT) * (NT / 64);
    return v > b ? v : b;
}

// b0: the blist0 array (player 0's bot PlayerAction: bot-vs-bot games, which are
// never bot-fused); wall: the terrain array (the fused step keeps it apart, at
// fb_wall_offset)
__host__ __device__ inline size_t lds_bytes(int HW, int W, int NT, bool b0 = true, bool wall = true) {
    size_t b = 0;
    b += a16(4 * (size_t)HW) * (b0 ? 10 : 9); // unit uid act seq aux resv list prod blist [blist0]
    b += a16(16 * (size_t)HW);     // snap
    b += wall ? a16((size_t)HW) : 0;
    b += a16(8 * (size_t)((HW + NT - 1) / NT) * (NT / 64) + 8);
    b += a16(4 * (size_t)((HW + 2 * W + 31) / 32 + 1));
    b += a16(4 * SC_WORDS);
    b += a16(vis_bytes(HW, NT));
    b += a16(8 * (size_t)((HW + 2 * W) / 32 + 1));
    return b;
}

// Bot-fused k_step layout (24x24 52.3 KB -> 40.1 KB, 3 -> 4
// workgroups per CU):
//   [0, core)   the step's arrays (no blist0, no terrain) until phase A, the
//               bot's (unit uid act ucell uuid pa, abstract actions) afterwards
//   outw        a bot game's output words: it streams them while wave 0 runs the
//               bot, so they lie outside the bot's region -- its mask words (one
//               view, 12 B per cell) here, its one-hot words (4 B per cell) in the
//               step's uid array on the early path (the bot reads uids only in its
//               setup, which the workgroup builds before the waves split), else
//               here behind the mask words
//   tail        the bot's small arrays (pend pab vis sc fw)
//   counter     the streaming waves' phase-A meeting point (early path)
//   wall        the terrain, read in place by the step, phase A and the bot
// Selfplay games of a fused launch run no bot and alias their output words onto
// the step's dead arrays, as the unfused kernel does.  `early`: the engine takes
// the early path (full observability and early_bot_disjoint).
__host__ __device__ inline size_t fb_outw_offset(int HW, int W, int NT) {
    const size_t a = lds_bytes(HW, W, NT, false, false), b = bots::bot_core_bytes(HW);
    return a16(a > b ? a : b);
}
__host__ __device__ inline size_t fb_tail_offset(int HW, int W, int NT, bool early) {
    return fb_outw_offset(HW, W, NT) + a16((early ? 12 : 16) * (size_t)HW);
}
__host__ __device__ inline size_t fb_early_cnt_offset(int HW, int W, int NT, bool early) {
    return fb_tail_offset(HW, W, NT, early) + a16(bots::bot_tail_bytes(HW, W));
}
__host__ __device__ inline size_t fb_wall_offset(int HW, int W, int NT, bool early) { return fb_early_cnt_offset(HW, W, NT, early) + 16; }
__host__ __device__ inline size_t fb_lds_bytes(int HW, int W, int NT, bool early) {
    return fb_wall_offset(HW, W, NT, early) + a16((size_t)HW);
}

__host__ __device__ inline Lds carve(unsigned char* base, int HW, int W, int NT, bool b0 = true, uint8_t* wall = nullptr) {
    Lds L;
    size_t o = 0;
    auto take = [&](size_t n) { unsigned char* p = base + o; o += a16(n); return p; };
    L.unit = (uint32_t*)take(4 * (size_t)HW);
    L.uid = (int32_t*)take(4 * (size_t)HW);
    L.act = (uint32_t*)take(4 * (size_t)HW);
    L.seq = (uint32_t*)take(4 * (size_t)HW);
    L.aux = (uint32_t*)take(4 * (size_t)HW);
    L.resv = (int32_t*)take(4 * (size_t)HW);
    L.list = (int32_t*)take(4 * (size_t)HW);
    L.prod = (int32_t*)take(4 * (size_t)HW);
    L.blist = (int32_t*)take(4 * (size_t)HW);
    // (!b0: unreachable by construction -- fused engines have no player-0 bots, mrts_capi fused())
    L.blist0 = b0 ? (int32_t*)take(4 * (size_t)HW) : L.blist;
    L.snap = (int4*)take(16 * (size_t)HW);
    L.outw = (uint32_t*)L.resv;   // resv, list, prod, blist, [blist0,] snap: >= 32 B per cell, contiguous
    L.outm = L.outw + 2 * HW;
    L.wall = wall ? wall : (uint8_t*)take((size_t)HW);
    L.ballot = (unsigned long long*)take(8 * (size_t)((HW + NT - 1) / NT) * (NT / 64) + 8);
    L.posbits = (uint32_t*)take(4 * (size_t)((HW + 2 * W + 31) / 32 + 1));
    L.sc = (int*)take(4 * SC_WORDS);
    L.vis = (uint32_t*)take(vis_bytes(HW, NT));
    L.claim = (uint32_t*)take(8 * (size_t)((HW + 2 * W) / 32 + 1));
    return L;
}

// The early-bot k_step (FB, P == 29): while wave 0 runs bots::bot_game (its
// small arrays in the tail region, the step's terrain read in place, setup
// preset), waves 1.. run emit_outputs' phase A, which reads the step's unit / act
// / wall / scalars and writes the output words (one-hot into the uid array, mask
// words behind the bot's region) and the meeting counter.  True when, for this
// map size, the bot writes none of those bytes and phase A writes none the bot
// reads -- computed from the two carves themselves -- and the bot's unit / uid /
// act arrays are the step's (it reads the state just stored in place).  The host
// takes the early path only then (EngineParams::early_bot; mrts_fused_layout_ok).
__host__ __device__ inline bool early_bot_disjoint(int HW, int W, int NT) {
    unsigned char* const z = reinterpret_cast<unsigned char*>((size_t)1 << 20);   // any base: only offsets matter
    const Lds S = carve(z, HW, W, NT, false, z + fb_wall_offset(HW, W, NT, true));
    const bots::BL B = bots::bot_carve(z, HW, W, z + fb_tail_offset(HW, W, NT, true), false);
    struct R {
        const void* p;
        size_t n;
    };
    auto lo = [&](const R& r) { return (size_t)((const unsigned char*)r.p - z); };
    auto overlap = [&](const R& a, const R& b) { return lo(a) < lo(b) + b.n && lo(b) < lo(a) + a.n; };
    const size_t hw = (size_t)HW, posw = (size_t)(HW + 2 * W) / 32 + 1, visw = (size_t)HW / 32 + 1;
    if (B.unit != S.unit || B.uid != S.uid || B.act != S.act) return false;
    const R bot_w[9] = {{B.ucell, 4 * hw}, {B.uuid, 4 * hw}, {B.pa, 4 * hw}, {B.aa, 32 * hw},
                        {B.pend, 4 * posw}, {B.pab, 4 * posw}, {B.vis, 4 * visw}, {B.sc, 16},
                        {B.fw, 4 * bots::bot_fw_words(HW)}};
    const R bot_r[3] = {{B.unit, 4 * hw}, {B.act, 4 * hw}, {S.wall, hw}};   // (uids: read by the setup only)
    const R a_r[3] = {{S.unit, 4 * hw}, {S.act, 4 * hw}, {S.wall, hw}};      // (resources: in registers)
    const R a_w[3] = {{S.uid, 4 * hw}, {z + fb_outw_offset(HW, W, NT), 12 * hw}, {z + fb_early_cnt_offset(HW, W, NT, true), 4}};
    for (const R& b : bot_w) {
        if (lo(b) + b.n > fb_lds_bytes(HW, W, NT, true)) return false;
        for (const R& a : a_r) if (overlap(a, b)) return false;
        for (const R& a : a_w) if (overlap(a, b)) return false;
    }
    for (const R& a : a_w)
        for (const R& b : bot_r) if (overlap(a, b)) return false;
    return true;
}

// Ordered block-wide compaction: list <- cells c (ascending) with pred(c);
// put(position, c) is called for every entry as it is written.  TAIL = false
// drops the trailing barrier: the caller orders the list before its readers, and
// the next compaction must use another s_mask.
struct NoPut {
    __device__ void operator()(int, int) const {}
};
template <int NT, bool TAIL = true, typename F, typename G = NoPut>
__device__ __forceinline__ int compact_cells(int HW, F pred, int32_t* list, unsigned long long* s_mask, G put = G()) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int J = (HW + NT - 1) / NT;
    for (int j = 0; j < J; j++) {
        int c = j * NT + threadIdx.x;
        bool f = c < HW && pred(c);
        unsigned long long m = __ballot(f);
        if (lane == 0) s_mask[j * NW + w] = m;
    }
    __syncthreads();
    int total = 0;
    for (int j = 0; j < J; j++) {
        int mi = j * NW + w;
        int before = 0;
        for (int k = 0; k < J * NW; k++) {
            int pc = __popcll(s_mask[k]);
            if (k < mi) before += pc;
            if (j == 0) total += pc;
        }
        unsigned long long m = s_mask[mi];
        if ((m >> lane) & 1ull) {
            const int pos = before + __popcll(m & ((1ull << lane) - 1ull)), c = j * NT + threadIdx.x;
            list[pos] = c;
            put(pos, c);
        }
    }
    if (TAIL) __syncthreads();
    return total;
}

// The early bot's setup, by the whole workgroup (all NT lanes, the state final
// in LDS, before the waves split): the parts of bots::bot_game's setup that are
// per cell -- the pending assignments' reservations and produce costs
// (isUnitActionAllowed's ResourceUsage), the free-cell words of path finding, and
// the unit list in pgs.units order (appended in any order, then ranked by uid)
// -- into the bot's LDS arrays (its tail zeroed at the kernel's start); the bot
// wave then starts at the abstract actions (bot_game, preset).  Full observability
// only (the early path's condition), so the bot's view is the state itself.
template <int NT>
__device__ __forceinline__ void bot_setup_workgroup(const EngineParams& p, unsigned char* smem, unsigned char* tail,
                                                    const uint8_t* wall) {
    const int HW = p.HW, W = p.W, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bots::BL B = bots::bot_carve(smem, HW, W, tail, false);
    // unit list by cell (B.pa), its uids alongside (the first words of B.aa, rewritten
    // by the bot later); B.sc[3] (zeroed with the tail) counts them
    int32_t* const ucells = B.pa;
    int32_t* const uids = reinterpret_cast<int32_t*>(B.aa);
    for (int base = 0; base < HW; base += NT) {
        const int c = base + (int)threadIdx.x;
        bool fr = false;
        if (c < HW) {
            const uint32_t u = B.unit[c], a = B.act[c];
            fr = !wall[c] && u == 0;
            if (u != 0) {
                const int pos = atomicAdd(&B.sc[3], 1);
                ucells[pos] = c;
                uids[pos] = B.uid[c];
            }
            if (a) {
                const int code = act_code(a), t = code_type(code);
                if (t == A_MOVE || t == A_PRODUCE) {
                    const int d = code_param(code), pos = c + (d == 0 ? -W : d == 1 ? 1 : d == 2 ? W : -1) + W;
                    atomicOr(&B.pend[pos >> 5], 1u << (pos & 31));
                    if (t == A_PRODUCE && u_owner(u) >= 0) atomicAdd(&B.sc[u_owner(u)], ut_cost(code_utype(code)));
                }
            }
        }
        const unsigned long long m = __ballot(fr);   // cells base + 64 wv .. + 63
        if (lane == 0 && base + 64 * wv < HW) {
            B.fw[(base + 64 * wv) / 32] = (uint32_t)m;
            B.fw[(base + 64 * wv) / 32 + 1] = (uint32_t)(m >> 32);
        }
    }
    __syncthreads();
    const int n = B.sc[3];
    for (int i = threadIdx.x; i < n; i += NT) {   // rank by uid (uids are unique)
        const int u = uids[i];
        int r = 0, j = 0;
        for (; j + 4 <= n; j += 4) {
            const int4 v = *reinterpret_cast<const int4*>(uids + j);
            r += (v.x < u) + (v.y < u) + (v.z < u) + (v.w < u);
        }
        for (; j < n; j++) r += uids[j] < u;
        B.ucell[r] = ucells[i];
        B.uuid[r] = u;
    }
}

struct Game {
    int g, env0, nviews, selfplay;
};
__device__ __forceinline__ Game game_of(const EngineParams& p, int g) {
    Game G;
    G.g = g;
    G.selfplay = g < p.nsp_games;
    G.env0 = G.selfplay ? 2 * g : p.nsp + (g - p.nsp_games);
    G.nviews = G.selfplay ? 2 : 1;
    return G;
}

// PhysicalGameState.load + new GameState into LDS
template <int NT>
__device__ __forceinline__ void reset_into_lds(const EngineParams& p, const Lds& L, int map) {
    const int HW = p.HW;
    for (int c = threadIdx.x; c < HW; c += NT) {
        int4 v = p.map_cells[(size_t)map * HW + c];
        L.unit[c] = (uint32_t)v.x;
        L.uid[c] = v.y;
        L.act[c] = 0;
        L.seq[c] = 0;
        L.wall[c] = p.map_wall[(size_t)map * HW + c];
    }
    if (threadIdx.x == 0) {
        const int* ms = p.map_scal + (size_t)map * MRTS_MAP_SCALARS;
        L.sc[SC_TIME] = 0;
        L.sc[SC_RES0] = ms[MRTS_M_RES0];
        L.sc[SC_RES1] = ms[MRTS_M_RES1];
        L.sc[SC_UID] = ms[MRTS_M_NUNITS];
        L.sc[SC_STEPS] = 0;
        L.sc[SC_MAP] = map;
    }
}

template <int NT>
__device__ __forceinline__ void load_game(const EngineParams& p, const Lds& L, int g) {
    if (threadIdx.x < MRTS_GENV_WORDS) L.sc[threadIdx.x] = p.genv[(size_t)g * MRTS_GENV_WORDS + threadIdx.x];
    __syncthreads();
    const int HW = p.HW, map = L.sc[SC_MAP];
    const int4* src = p.cells + (size_t)g * p.cstride;
    for (int c = threadIdx.x; c < HW; c += NT) {
        int4 v = src[c];
        L.unit[c] = (uint32_t)v.x;
        L.uid[c] = v.y;
        L.act[c] = (uint32_t)v.z;
        L.seq[c] = (uint32_t)v.w;
        L.wall[c] = p.map_wall[(size_t)map * HW + c];
    }
    __syncthreads();
}

template <int NT>
__device__ __forceinline__ void store_game(const EngineParams& p, const Lds& L, int g) {
    const int HW = p.HW;
    int4* dst = p.cells + (size_t)g * p.cstride;
    for (int c = threadIdx.x; c < HW; c += NT) dst[c] = make_int4((int)L.unit[c], L.uid[c], (int)L.act[c], (int)L.seq[c]);
    if (threadIdx.x < MRTS_GENV_WORDS) p.genv[(size_t)g * MRTS_GENV_WORDS + threadIdx.x] = L.sc[threadIdx.x];
}

// PartiallyObservableGameState.observable for both players: a cell is seen by
// player q when some unit of q is within its sight radius (d^2 <= r^2).  Each
// unit lane ORs its sight disk into the player's LDS bitmap, one row span per
// atomic (or_sight_disk).
template <int NT>
__device__ __forceinline__ void compute_vis(const EngineParams& p, const Lds& L) {
    const int HW = p.HW, nw = HW / 32 + 1;
    for (int i = threadIdx.x; i < 2 * nw; i += NT) L.vis[i] = 0;
    __syncthreads();
    for (int c = threadIdx.x; c < HW; c += NT) {
        uint32_t u = L.unit[c];
        int q = u_owner(u);
        if (u == 0 || q < 0) continue;
        or_sight_disk(L.vis + q * nw, c % p.W, c / p.W, ut_sight(u_type(u)), p.W, p.H);
    }
    __syncthreads();
}

// phase A's one-hot word of cell c for every view of the game (into L.outw)
template <int P>
__device__ __forceinline__ void onehot_words(const EngineParams& p, const Lds& L, const Game& G, int c) {
    const int HW = p.HW, nw = HW / 32 + 1;
    const uint32_t u = L.unit[c], a = L.act[c];
    const uint8_t wl = L.wall[c];
    for (int v = 0; v < G.nviews; v++) {
        if (P == 31) {
            const bool shown = u == 0 || u_owner(u) == v || ((L.vis[v * nw + (c >> 5)] >> (c & 31)) & 1u);
            const bool opp = (L.vis[(1 - v) * nw + (c >> 5)] >> (c & 31)) & 1u;
            L.outw[v * HW + c] = cell_onehot(u, a, wl, v, P, shown, opp);
        } else {
            L.outw[v * HW + c] = cell_onehot(u, a, wl, v);
        }
    }
}
__device__ __forceinline__ void mask_words(const EngineParams& p, const Lds& L, const Game& G, int c, int res0, int res1) {
    const int HW = p.HW;
    const Grid gd{p.W, p.H, HW};
    for (int v = 0; v < G.nviews; v++) {
        uint32_t m[3];
        cell_mask(gd, c, v, L.unit, L.act, L.wall, v == 0 ? res0 : res1, m);
        L.outm[3 * (v * HW + c)] = m[0];
        L.outm[3 * (v * HW + c) + 1] = m[1];
        L.outm[3 * (v * HW + c) + 2] = m[2];
        p.src_out[(size_t)(G.env0 + v) * HW + c] = (int32_t)(m[0] & 1u);
    }
}
// phase B's obs rows of every view, lanes t0 .. t0 + nt
template <int P, typename OT>
__device__ __forceinline__ void stream_obs(const EngineParams& p, const Lds& L, const Game& G, int t0, int nt) {
    const int HW = p.HW, NV = G.nviews;
    const uint32_t* ow = L.outw;
    OT* out = reinterpret_cast<OT*>(p.obs) + (size_t)G.env0 * HW * P;
    const int total = NV * HW * P;
    if (((HW * P) & 3) == 0) {   // every env's rows start 16-B aligned
        constexpr int ONE = std::is_same<OT, float>::value ? 0x3f800000 : 1;   // 1.0f or 1 as stored bits
        // elements e .. e+3 are planes pl .. pl+3 of cell c, running on into cell
        // c+1 past plane P-1: one paired LDS read (cells c, c+1) per 16-B store.
        // (c+1 past the last cell reads the words behind: never used, as the last
        // store of the run ends at plane P-1.)  A one-hot word has no bit at or
        // above P, so (w0 >> pl) | (w1 << (P - pl)) are the window's bits.  (c, pl)
        // advance by a constant per trip: no division in the loop.
        // Software-pipelined: the next trip's word pair is read before this trip's
        // store, so the LDS round trip overlaps the bit work instead of stalling every
        // trip (a lone workgroup's stream -- the kernel's last round -- is bound by this
        // loop, not by the store path: scripts/store_rate.hip).  The read-ahead index is
        // clamped into the word region (its last trip's values are never used).
        const int dq = 4 * nt / P, dr = 4 * nt - dq * P, cmax = NV * HW - 1;
        int c = 4 * t0 / P, pl = 4 * t0 - c * P;
        uint32_t w0 = ow[min(c, cmax)], w1 = ow[min(c, cmax) + 1];
        for (int k = t0; k < total / 4; k += nt) {
            int cn = c + dq, pn = pl + dr;
            if (pn >= P) { pn -= P; cn++; }
            const int cr = min(cn, cmax);
            const uint32_t n0 = ow[cr], n1 = ow[cr + 1];
            const uint32_t bits = (w0 >> pl) | (w1 << (P - pl));
            st16(out + 4 * k, (bits & 1u) ? ONE : 0, (bits & 2u) ? ONE : 0, (bits & 4u) ? ONE : 0, (bits & 8u) ? ONE : 0);
            w0 = n0;
            w1 = n1;
            c = cn;
            pl = pn;
        }
    } else {
        for (int e = t0; e < total; e += nt) out[e] = (OT)((ow[e / P] >> (e % P)) & 1u);
    }
}
// phase B's mask rows of every view, lanes t0 .. t0 + nt
__device__ __forceinline__ void stream_masks(const EngineParams& p, const Lds& L, const Game& G, int t0, int nt) {
    const int HW = p.HW, NV = G.nviews;
    const uint32_t* mw = L.outm;
    int32_t* out = p.mask + (size_t)G.env0 * HW * MRTS_MASK_CH;
    const int total = NV * HW * MRTS_MASK_CH;
    if ((HW & 1) == 0) {   // HW * 78 % 4 == 0: every env's rows start 16-B aligned
        // elements e .. e+3 are channels ch .. ch+3 of row r = bits ch+1 .. ch+4 of
        // its 79-bit word (bit 0 = source); e is a multiple of 4 and a row pair
        // is 156 elements, so ch is even and only ch = 76 runs into row r+1
        // (channels 76, 77 = bits 77, 78, then bits 1, 2 of the next row, whose
        // first word is the word after bit 78's).  One paired LDS read per store.
        // (r, ch) advance by a constant per trip; the ch == 76 fix-up is a select,
        // not a branch.
        static_assert(MRTS_MASK_CH == 78, "mask row layout");
        // (software-pipelined as the obs loop: the next trip's word pair read ahead)
        const int dq = 4 * nt / MRTS_MASK_CH, dr = 4 * nt - dq * MRTS_MASK_CH, wmax = 3 * NV * HW - 1;
        int r = 4 * t0 / MRTS_MASK_CH, ch = 4 * t0 - r * MRTS_MASK_CH;
        int r3 = 3 * r;   // the row's first word
        int wr = min(r3 + ((ch + 1) >> 5), wmax);
        uint32_t lo = mw[wr], hi = mw[wr + 1];
        for (int k = t0; k < total / 4; k += nt) {
            int r3n = r3 + 3 * dq, chn = ch + dr;
            if (chn >= MRTS_MASK_CH) { chn -= MRTS_MASK_CH; r3n += 3; }
            wr = min(r3n + ((chn + 1) >> 5), wmax);
            const uint32_t nlo = mw[wr], nhi = mw[wr + 1];
            const int b0 = ch + 1;
            const uint32_t fun = (uint32_t)((((uint64_t)hi << 32) | lo) >> (b0 & 31));
            const uint32_t bits = ch == 76 ? ((fun & 3u) | ((hi << 1) & 0xCu)) : fun;
            st16(out + 4 * k, (int)(bits & 1u), (int)((bits >> 1) & 1u), (int)((bits >> 2) & 1u), (int)((bits >> 3) & 1u));
            lo = nlo;
            hi = nhi;
            r3 = r3n;
            ch = chn;
        }
    } else {
        for (int e = t0; e < total; e += nt) {
            const int r = e / MRTS_MASK_CH, b = e % MRTS_MASK_CH + 1;
            out[e] = (int)((mw[3 * r + (b >> 5)] >> (b & 31)) & 1u);
        }
    }
}

// All outputs of one game once its state is final.  Phase A (lane per cell):
// every view's one-hot word and, with `masks`, its getMasks(0) 79-bit word
// (+ the source channel, written straight out) into LDS; one barrier; phase B:
// the views' obs rows, then their mask rows, streamed with 16-byte stores and no
// further barrier (the envs of a game are adjacent: a selfplay pair 2k, 2k+1
// writes one contiguous run).  The words live in the region of the step's
// scratch lists (resv .. snap), dead by now.
// `skip`: lanes [0, skip) leave after phase A (the bot-fused k_step's wave 0) and
// the others stream phase B alone.
// `early_cnt` (the early-bot k_step): wave 0 is running the bot already, so
// phase A too runs on lanes [skip, NT) only and its end is a counter the
// streaming waves meet at in LDS instead of a workgroup barrier.
// res0 / res1: the players' resources (the masks' produce checks), read by the
// caller from L.sc before the early bot may overwrite the step's scalars.
// Masks first (no bot in the workgroup, skip == 0): the mask words (no fog
// dependency) are built and their 2.5x larger stream issued before the one-hot
// words (and, under partial observability, the sight disks) are computed, so a
// game's first bytes leave one phase earlier and the obs words are built while the
// mask stores drain; one more barrier before the obs stream.
template <int NT, int P, typename OT>
__device__ __forceinline__ void emit_outputs(const EngineParams& p, const Lds& L, const Game& G, bool obs, bool masks, int res0,
                                             int res1, int skip = 0, int* early_cnt = nullptr) {
    const int HW = p.HW;
    if (skip == 0 && obs && masks) {
        const int nw = HW / 32 + 1;
        for (int c = threadIdx.x; c < HW; c += NT) mask_words(p, L, G, c, res0, res1);
        if (P == 31)
            for (int i = threadIdx.x; i < 2 * nw; i += NT) L.vis[i] = 0;
        __syncthreads();
        MRTS_STAMP(8, threadIdx.x == 0);
        __builtin_amdgcn_s_setprio(0);
        stream_masks(p, L, G, threadIdx.x, NT);
        if (P == 31) {   // compute_vis's sight disks (cleared above)
            for (int c = threadIdx.x; c < HW; c += NT) {
                const uint32_t u = L.unit[c];
                const int q = u_owner(u);
                if (u != 0 && q >= 0) or_sight_disk(L.vis + q * nw, c % p.W, c / p.W, ut_sight(u_type(u)), p.W, p.H);
            }
            __syncthreads();
        }
        for (int c = threadIdx.x; c < HW; c += NT) onehot_words<P>(p, L, G, c);
        __syncthreads();
        stream_obs<P, OT>(p, L, G, threadIdx.x, NT);
        MRTS_STAMP_MAX(9, (threadIdx.x & 63) == 0);
        return;
    }
    if (obs && P == 31) compute_vis<NT>(p, L);
    const int a0 = early_cnt ? skip : 0;   // phase A's first lane
    for (int c = (int)threadIdx.x - a0; c < HW; c += NT - a0) {
        if (obs) onehot_words<P>(p, L, G, c);
        if (masks) mask_words(p, L, G, c, res0, res1);
    }
    if (early_cnt) {   // the streaming waves' own meeting point (wave 0 never arrives)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if ((threadIdx.x & 63u) == 0) __hip_atomic_fetch_add(early_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(early_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (NT - skip) / 64)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __syncthreads();
    }
    // ---- phase B -----------------------------------------------------------
    // Bot-fused k_step (skip = 64): from here on wave 0 runs bots::bot_game, whose
    // LDS region starts at smem offset 0 and overwrites the step's arrays but the
    // unit / act / wall it reads and, on the early path, the uid array.  Phase B
    // must read nothing but the output words `ow` / `mw` (fb_outw_offset) and
    // kernel parameters.
    if ((int)threadIdx.x < skip) return;
    MRTS_STAMP(8, (int)threadIdx.x == skip);
    __builtin_amdgcn_s_setprio(0);
    const int t0 = (int)threadIdx.x - skip, nt = NT - skip;
    if (obs) stream_obs<P, OT>(p, L, G, t0, nt);
    if (masks) stream_masks(p, L, G, t0, nt);
    MRTS_STAMP_MAX(9, (threadIdx.x & 63) == 0);
}

// A parked game's envs read zero: mask / source rows (when p.mask is set), and
// obs rows (zero_outputs).
template <int NT>
__device__ __forceinline__ void zero_mask_rows(const EngineParams& p, const Game& G) {
    if (!p.mask) return;
    const size_t n = (size_t)G.nviews * p.HW;
    int32_t* m = p.mask + (size_t)G.env0 * p.HW * MRTS_MASK_CH;
    for (size_t i = threadIdx.x; i < n * MRTS_MASK_CH; i += NT) m[i] = 0;
    for (size_t i = threadIdx.x; i < n; i += NT) p.src_out[(size_t)G.env0 * p.HW + i] = 0;
}
template <int NT, int P, typename OT>
__device__ __forceinline__ void zero_outputs(const EngineParams& p, const Game& G) {
    const size_t n = (size_t)G.nviews * p.HW;
    OT* obs = reinterpret_cast<OT*>(p.obs) + (size_t)G.env0 * p.HW * P;
    for (size_t i = threadIdx.x; i < n * P; i += NT) obs[i] = (OT)0;
    zero_mask_rows<NT>(p, G);
}

// ---------------------------------------------------------------------------
// Reset kernel: every game (or the listed ones) back to its map; obs out.
// Parked games (mrts_park_games) keep their state and write zero outputs.
template <int NT, int P, typename OT>
__global__ __launch_bounds__(NT) void k_reset(EngineParams p, const int32_t* games, const int32_t* maps, int count) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MRTS_STAMP_NONE();
    Lds L = carve(smem, p.HW, p.W, NT);
    int g = games ? games[blockIdx.x] : blockIdx.x;
    if (game_parked(p, g)) {
        zero_outputs<NT, P, OT>(p, game_of(p, g));
        return;
    }
    int map = maps ? maps[blockIdx.x] : p.genv[(size_t)g * MRTS_GENV_WORDS + MRTS_G_MAP];
    // a reset keeps the never-reset counters (bot RNG ticks, rollout statistics)
    if (threadIdx.x < SC_WORDS) {
        const int w = threadIdx.x;
        const bool keep = w == SC_TICKS || w == MRTS_G_SERIAL || w == MRTS_G_ORDERED || w == MRTS_G_EPISODES;
        L.sc[w] = keep ? p.genv[(size_t)g * MRTS_GENV_WORDS + w] : 0;
    }
    __syncthreads();
    reset_into_lds<NT>(p, L, map);
    __syncthreads();
    store_game<NT>(p, L, g);
    Game G = game_of(p, g);
    emit_outputs<NT, P, OT>(p, L, G, true, p.mask != nullptr, L.sc[SC_RES0], L.sc[SC_RES1]);
}

// ---------------------------------------------------------------------------
// Raw observation kernel: Response.observation = GameState.getVectorObservation
// (player) as the JNI client returns it, int32 [N][P_raw][H][W] (P_raw = 6, or 7
// with partial obs) -- the input of the reference's python _encode_obs
// (vec_env.py:280, 1035).  Same per-cell rules as cell_onehot, unencoded.
template <int NT>
__global__ __launch_bounds__(NT) void k_raw(EngineParams p, int32_t* raw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Lds L = carve(smem, p.HW, p.W, NT);
    const int g = blockIdx.x, HW = p.HW;
    const Game G = game_of(p, g);
    const int PR = p.partial_obs ? 7 : 6, nw = HW / 32 + 1;
    if (game_parked(p, g)) {   // a parked game's envs read zero (mrts_park_games)
        int32_t* out = raw + (size_t)G.env0 * PR * HW;
        for (int i = threadIdx.x; i < G.nviews * PR * HW; i += NT) out[i] = 0;
        return;
    }
    load_game<NT>(p, L, g);
    if (p.partial_obs) compute_vis<NT>(p, L);
    for (int v = 0; v < G.nviews; v++) {
        int32_t* out = raw + (size_t)(G.env0 + v) * PR * HW;
        for (int c = threadIdx.x; c < HW; c += NT) {
            uint32_t u = L.unit[c], a = L.act[c];
            if (p.partial_obs && u != 0 && u_owner(u) != v && !((L.vis[v * nw + (c >> 5)] >> (c & 31)) & 1u)) u = 0;
            const int ow = u_owner(u);
            out[0 * HW + c] = u ? u_hp(u) : 0;
            out[1 * HW + c] = u ? u_res(u) : 0;
            out[2 * HW + c] = (u && ow >= 0) ? (ow == v ? 1 : 2) : 0;
            out[3 * HW + c] = u ? u_type(u) + 1 : 0;
            out[4 * HW + c] = (u && a) ? code_type(act_code(a)) : 0;
            out[5 * HW + c] = L.wall[c];
            if (p.partial_obs) out[6 * HW + c] = (u && ((L.vis[(1 - v) * nw + (c >> 5)] >> (c & 31)) & 1u)) ? 1 : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// Mask kernel: JNIGridnetVecClient.getMasks(0) -> [N][HW][78] + source [N][HW]
template <int NT>
__global__ __launch_bounds__(NT) void k_masks(EngineParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MRTS_STAMP_NONE();
    Lds L = carve(smem, p.HW, p.W, NT);
    const int g = blockIdx.x;
    if (game_parked(p, g)) {   // the caller's buffers need not be the ones zeroed at park time
        zero_mask_rows<NT>(p, game_of(p, g));
        return;
    }
    load_game<NT>(p, L, g);
    emit_outputs<NT, 29, int32_t>(p, L, game_of(p, g), false, true, L.sc[SC_RES0], L.sc[SC_RES1]);
}

// ---------------------------------------------------------------------------
// Outputs kernel: the obs (and, when bound, the next-tick masks) of every game's
// stored state, unchanged -- after an env-state checkpoint is restored
// (mrts_load_state).  Parked games read zero.
template <int NT, int P, typename OT>
__global__ __launch_bounds__(NT) void k_outputs(EngineParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MRTS_STAMP_NONE();
    Lds L = carve(smem, p.HW, p.W, NT);
    const int g = blockIdx.x;
    if (game_parked(p, g)) {
        zero_outputs<NT, P, OT>(p, game_of(p, g));
        return;
    }
    load_game<NT>(p, L, g);
    emit_outputs<NT, P, OT>(p, L, game_of(p, g), true, p.mask != nullptr, L.sc[SC_RES0], L.sc[SC_RES1]);
}

// ---------------------------------------------------------------------------
// Step kernel: JNIGridnetVecClient.gameStep for one game per workgroup.
enum : uint32_t { CAND = 1u << 31, LEGAL = 1u << 30 };
__device__ __forceinline__ int unchecked_pos(const Grid& gd, int c, int dir) {   // UnitAction.resourceUsage position
    const int off[4] = {-gd.W, 1, gd.W, -1};
    return c + off[dir];
}

__device__ __forceinline__ int res_of(const Lds& L, int player) { return L.sc[SC_RES0 + player]; }

// Step (2a)'s target-position claims of a move / produce row: bit b of claim[0..posw)
// when >= 1 row targets position b (x + y * W + W, unchecked), of claim[posw..) when >= 2.
__device__ __forceinline__ void claim_target(const Lds& L, const Grid& gd, int c, int code, int posw) {
    const int ty = code_type(code);
    if (ty != A_MOVE && ty != A_PRODUCE) return;
    const int b = unchecked_pos(gd, c, code_param(code)) + gd.W;
    const uint32_t bit = 1u << (b & 31);
    if (atomicOr(&L.claim[b >> 5], bit) & bit) atomicOr(&L.claim[posw + (b >> 5)], bit);
}

// PlayerAction.fromVectorAction consistency filter + GameState.issueSafe/issue
// for one player's PlayerAction (lane 0 only).  Entries are list[0..n) in
// PlayerAction order with their codes in L.aux: the agent's rows (ascending
// cells, `vector` = true: the fromVectorAction consistency filter applies and
// the LinkedHashMap rank is the cell) or a device bot's PlayerAction (already
// consistent, rank = position in the list).
__device__ __forceinline__ void issue_player(const EngineParams& p, const Lds& L, const Grid& gd, int q, const int32_t* list, int n,
                             bool vector) {
    const int time = L.sc[SC_TIME];
    // --- fromVectorAction: ResourceUsage.consistentWith(pa.ru) ----------------
    const int nposw = (gd.HW + 2 * gd.W + 31) / 32;
    for (int i = 0; i < nposw; i++) L.posbits[i] = 0;
    int pa_cost = 0;
    for (int i = 0; vector && i < n; i++) {
        int c = list[i];
        uint32_t nw = L.aux[c];
        if (u_owner(L.unit[c]) != q) continue;
        int code = (int)(nw & 0xFFFu), type = code_type(code);
        if (type != A_MOVE && type != A_PRODUCE) continue;
        const int off[4] = {-gd.W, 1, gd.W, -1};
        int pos = c + off[code_param(code)];   // unchecked, as x + y*W + offset
        int cost = type == A_PRODUCE ? ut_cost(code_utype(code)) : 0;
        int bi = pos + gd.W;
        bool taken = (L.posbits[bi >> 5] >> (bi & 31)) & 1u;
        int s = cost + pa_cost;
        if (taken || (s > 0 && s > res_of(L, q))) {
            L.aux[c] = nw & ~CAND;   // dropped: gets fillWithNones
            continue;
        }
        L.posbits[bi >> 5] |= 1u << (bi & 31);
        pa_cost += cost;
    }
    // --- issueSafe + issue -----------------------------------------------------
    int* rw = L.sc + SC_R0 + 6 * q;
    for (int i = 0; i < n; i++) {
        int c = list[i];
        uint32_t nw = L.aux[c];
        if (u_owner(L.unit[c]) != q || !(nw & CAND)) continue;
        const int ut = u_type(L.unit[c]);
        int code = (int)(nw & 0xFFFu);
        // issueSafe: illegal -> NONE with the same ETA
        int cur = code, cur_dur = 1;   // cur_dur: duration when cur is NONE (a NONE code's param)
        if (code_type(code) == A_NONE) cur_dur = code_param(code);
        else if (!(nw & LEGAL)) { cur_dur = eta_code(code, ut); cur = A_NONE; }
        int te = cur;                  // the action the TraceEntry records
        const int ctype = code_type(cur);
        int pos = -1, cost_new = 0;
        if (ctype == A_MOVE || ctype == A_PRODUCE) pos = nb_cell(gd, c, code_param(cur));
        if (ctype == A_PRODUCE) cost_new = ut_cost(code_utype(cur));
        // uaa's inconsistent with the new ResourceUsage (the holder of the target
        // position, pending produces over a player's budget), visited in
        // LinkedHashMap order: each pass takes the candidate of least issue
        // sequence above the last one visited -- any number of candidates, no
        // buffer.  Visiting a candidate rewrites only its own action, and every
        // candidate is tested against its action before the visit, as in issue().
        const int nprod = L.sc[SC_NPROD];
        const int rc = (pos >= 0) ? L.resv[pos] : -1;
        bool original = true;
        uint32_t last = 0;
        for (bool first = true;; first = false) {
            int cc = -1;
            uint32_t best = 0xFFFFFFFFu;
            if (rc >= 0 && (first || L.seq[rc] > last) && L.seq[rc] < best) { cc = rc; best = L.seq[rc]; }
            for (int k = 0; k < nprod; k++) {
                const int pc = L.prod[k];
                const uint32_t sq = L.seq[pc];
                if (pc == rc || (!first && sq <= last) || sq >= best) continue;
                const uint32_t pa = L.act[pc];
                if (pa == 0 || code_type(act_code(pa)) != A_PRODUCE) continue;
                const int pp = u_owner(L.unit[pc]), cp = ut_cost(code_utype(act_code(pa)));
                bool bad = false;
                for (int pl = 0; pl < 2; pl++) {
                    const int s = (pp == pl ? cp : 0) + (q == pl ? cost_new : 0);
                    if (s > 0 && s > res_of(L, pl)) bad = true;
                }
                if (bad) { cc = pc; best = sq; }
            }
            if (cc < 0) break;
            last = best;
            uint32_t ua = L.act[cc];
            if (seq_time(L.seq[cc]) == time) {    // CANCEL_BOTH
                int ucode = act_code(ua);
                int d1 = eta_code(ucode, u_type(L.unit[cc]));
                int d2 = code_type(cur) == A_NONE ? cur_dur : eta_code(cur, ut);
                int d = min(d1, d2);
                int utp = code_type(ucode);
                if (utp == A_MOVE || utp == A_PRODUCE) {
                    int rp = nb_cell(gd, cc, code_param(ucode));
                    if (rp >= 0 && L.resv[rp] == cc) L.resv[rp] = -1;
                }
                L.act[cc] = act_make(A_NONE, time + d);
                cur = A_NONE;
                cur_dur = d;
                original = false;
            } else {                               // "Inconsistent actions were executed!"
                cur = A_NONE;
                cur_dur = -1;
                if (original) te = A_NONE;
            }
        }
        const int ft = code_type(cur);
        const int done = ft == A_NONE ? time + cur_dur : time + eta_code(cur, ut);
        L.act[c] = act_make(cur, done);
        L.seq[c] = seq_make(time, q, vector ? c : i);
        if (ft == A_MOVE || ft == A_PRODUCE) {
            L.resv[nb_cell(gd, c, code_param(cur))] = c;
            if (ft == A_PRODUCE) L.prod[L.sc[SC_NPROD]++] = c;
        }
        // ai.reward.* on the TraceEntry actions
        const int tt = code_type(te);
        if (tt == A_HARVEST || tt == A_RETURN) rw[1]++;
        if (tt == A_PRODUCE) {
            int pu = code_utype(te);
            if (pu == WORKER) rw[2]++;
            else if (pu == BASE || pu == BARRACKS) rw[3]++;
            else if (pu >= LIGHT) rw[5]++;
        }
        if (tt == A_ATTACK) rw[4]++;
    }
}

// UnitAction.execute for one ready assignment, from its snapshot.  Serial
// (lane 0, issue order) or, for an independent ready set, one lane per action
// (PAR: resource / error updates are atomic, the produced unit's id is given).
template <bool PAR = false>
__device__ __forceinline__ void execute_one(const Lds& L, const Grid& gd, int4 s, int produced_uid = -1) {
    const int c = s.x;
    const uint32_t u = (uint32_t)s.y;
    const int code = (int)(s.z);
    const int uid = s.w;
    const int t = u_type(u), owner = u_owner(u);
    const bool here = L.unit[c] != 0 && L.uid[c] == uid;   // not killed earlier this cycle
    const int type = code_type(code), param = code_param(code);
    switch (type) {
    case A_MOVE: {
        if (!here) break;
        int n = nb_cell(gd, c, param);
        if (n < 0 || L.unit[n] != 0) {
            if (PAR) atomicOr(&L.sc[SC_ERR], MRTS_ERR_MOVE_OCCUPIED);
            else L.sc[SC_ERR] |= MRTS_ERR_MOVE_OCCUPIED;
            break;
        }
        L.unit[n] = L.unit[c];
        L.uid[n] = uid;
        L.act[n] = 0;
        L.seq[n] = 0;
        L.unit[c] = 0;
        L.uid[c] = 0;
        L.act[c] = 0;
        L.seq[c] = 0;
        break;
    }
    case A_ATTACK: {
        int dx = param % MRTS_ATTACK_GRID - MRTS_ATTACK_GRID / 2, dy = param / MRTS_ATTACK_GRID - MRTS_ATTACK_GRID / 2;
        int x = c % gd.W + dx, y = c / gd.W + dy;
        if (x < 0 || y < 0 || x >= gd.W || y >= gd.H) break;
        int n = y * gd.W + x;
        uint32_t o = L.unit[n];
        if (o == 0) break;
        int hp = u_hp(o) - ut_damage(t);   // VERSION_ORIGINAL: min == max damage
        if (hp <= 0) {                     // GameState.removeUnit (+ its assignment)
            const int vo = u_owner(o);
            if (vo == 0 || vo == 1) {      // the players' unit counts (k_step's SC_HAS)
                if (PAR) atomicSub(&L.sc[SC_HAS], vo ? 1 << 16 : 1);
                else L.sc[SC_HAS] -= vo ? 1 << 16 : 1;
            }
            L.unit[n] = 0;
            L.uid[n] = 0;
            L.act[n] = 0;
            L.seq[n] = 0;
        } else {
            L.unit[n] = u_with_hp(o, hp);
        }
        break;
    }
    case A_HARVEST: {
        int n = nb_cell(gd, c, param);
        if (n < 0) break;
        uint32_t o = L.unit[n];
        if (o == 0 || u_type(o) != RESOURCE || !ut_can_harvest(t) || u_res(u) != 0) break;
        int left = u_res(o) - ut_harvest_amount(t);
        if (left <= 0) {
            L.unit[n] = 0;
            L.uid[n] = 0;
            L.act[n] = 0;
            L.seq[n] = 0;
        } else {
            L.unit[n] = u_with_res(o, left);
        }
        if (here) L.unit[c] = u_with_res(L.unit[c], ut_harvest_amount(t));
        break;
    }
    case A_RETURN: {
        int n = nb_cell(gd, c, param);
        if (n < 0) break;
        uint32_t o = L.unit[n];
        if (o == 0 || !ut_is_stockpile(u_type(o)) || u_res(u) <= 0) break;
        if (PAR) atomicAdd(&L.sc[SC_RES0 + owner], u_res(u));
        else L.sc[SC_RES0 + owner] += u_res(u);
        if (here) L.unit[c] = u_with_res(L.unit[c], 0);
        break;
    }
    case A_PRODUCE: {
        int n = nb_cell(gd, c, param);
        int put = code_utype(code);
        if (n < 0 || L.unit[n] != 0) {
            if (PAR) atomicOr(&L.sc[SC_ERR], MRTS_ERR_PRODUCE_OCCUPIED);
            else L.sc[SC_ERR] |= MRTS_ERR_PRODUCE_OCCUPIED;
            break;
        }
        L.unit[n] = u_make(put, owner, ut_hp(put), 0);
        L.uid[n] = PAR ? produced_uid : L.sc[SC_UID]++;
        if (owner == 0 || owner == 1) {
            if (PAR) atomicAdd(&L.sc[SC_HAS], owner ? 1 << 16 : 1);
            else L.sc[SC_HAS] += owner ? 1 << 16 : 1;
        }
        L.act[n] = 0;
        L.seq[n] = 0;
        if (PAR) atomicSub(&L.sc[SC_RES0 + owner], ut_cost(put));
        else L.sc[SC_RES0 + owner] -= ut_cost(put);
        break;
    }
    default: break;
    }
}

// Wider maps (NT < HW <= 4 NT, e.g. 24x24 and 32x32 on 256 lanes): the lane's
// cells, their source-unit words and the terrain in registers, all issued in one
// round trip with genv (the unprefetched path takes four: genv, cells, then the
// sources and the actions inside the decode); the source words reach the decode
// through L.aux.
struct WidePf {
    int4 cell[4];
    int src[4];   // bit v: the source-unit word of view v
    int wall[4];
    int genv, map;
    int bpa0, bpa1;   // bot games: entry `lane` of the bot PlayerActions (player 0 / 1)
};
template <int NT>
__device__ __forceinline__ void prefetch_wide(const EngineParams& p, const Game& G, int g, WidePf& pf) {
    const int HW = p.HW;
    pf.genv = p.genv[(size_t)g * MRTS_GENV_WORDS + min((int)threadIdx.x, MRTS_GENV_WORDS - 1)];
    pf.map = p.nmaps == 1 ? 0 : p.genv[(size_t)g * MRTS_GENV_WORDS + MRTS_G_MAP];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = min((int)threadIdx.x + k * NT, HW - 1);   // unconditional: counted waits
        pf.cell[k] = p.cells[(size_t)g * p.cstride + c];
        const int s0 = p.src[(size_t)G.env0 * HW + c], s1 = p.src[(size_t)(G.env0 + G.nviews - 1) * HW + c];
        pf.src[k] = (s0 ? 1 : 0) | (s1 ? 2 : 0);
        if (p.nmaps == 1) pf.wall[k] = p.map_wall[c];
    }
    if (!G.selfplay && p.botpa) {   // speculative: the counts arrive with genv
        const int32_t* bp = p.botpa + (size_t)(g - p.nsp_games) * 2 * HW;
        pf.bpa0 = p.bot_ai0 ? bp[threadIdx.x] : 0;
        pf.bpa1 = bp[HW + threadIdx.x];
    }
}
template <int NT>
__device__ __forceinline__ void commit_wide(const EngineParams& p, const Lds& L, const WidePf& pf) {
    if (threadIdx.x < MRTS_GENV_WORDS) L.sc[threadIdx.x] = pf.genv;
    const int HW = p.HW;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = (int)threadIdx.x + k * NT;
        if (c >= HW) break;
        L.unit[c] = (uint32_t)pf.cell[k].x;
        L.uid[c] = pf.cell[k].y;
        L.act[c] = (uint32_t)pf.cell[k].z;
        L.seq[c] = (uint32_t)pf.cell[k].w;
        L.wall[c] = p.nmaps == 1 ? (uint8_t)pf.wall[k] : p.map_wall[(size_t)pf.map * HW + c];
        L.resv[c] = -1;
        L.aux[c] = (uint32_t)pf.src[k];   // read back by the decode on this lane
    }
    __syncthreads();
}

// Register prefetch of a game's state (maps with HW <= NT: one cell per lane):
// issued before the current game's output stream, so the next game's state
// round trip overlaps those stores instead of stalling the block.
struct StatePf {
    int4 cell;
    int genv, src0, src1;
    int bpa0, bpa1;   // bot games: entry `lane` of the bot PlayerActions (player 0 / 1)
    int4 aa, aa2;     // bot-fused games, lanes < 64: words lane, lane + 64 of the bot's abstract actions
    int wall;         // single-map batches: this cell's terrain
    int map;          // the game's map (genv[MRTS_G_MAP], every lane: no barrier before the terrain load)
};
// the bot wave's first abstract-action words: lane, lane + 64 of the game's 2 * HW (clamped: small maps)
__device__ __forceinline__ void prefetch_aa(const EngineParams& p, int g, StatePf& pf) {
    const int4* aa = p.aa + ((size_t)(g - p.nsp_games) * 2 + 1) * p.HW * 2;
    pf.aa = aa[min((int)threadIdx.x, 2 * p.HW - 1)];
    pf.aa2 = aa[min(64 + (int)threadIdx.x, 2 * p.HW - 1)];
}
template <int NT, bool FB>
__device__ __forceinline__ void prefetch_game(const EngineParams& p, int g, StatePf& pf) {
    const Game G = game_of(p, g);
    const int HW = p.HW, c = min((int)threadIdx.x, HW - 1);   // unconditional: counted waits
    pf.cell = p.cells[(size_t)g * p.cstride + c];
    pf.src0 = p.src[(size_t)G.env0 * HW + c];
    pf.src1 = p.src[(size_t)(G.env0 + G.nviews - 1) * HW + c];
    pf.genv = p.genv[(size_t)g * MRTS_GENV_WORDS + min((int)threadIdx.x, MRTS_GENV_WORDS - 1)];
    if (!G.selfplay && p.botpa) {   // speculative: the counts arrive with genv
        const int32_t* bp = p.botpa + (size_t)(g - p.nsp_games) * 2 * HW;
        pf.bpa0 = p.bot_ai0 ? bp[c] : 0;   // player 0 bots: MicroRTSBotVecEnv only
        pf.bpa1 = bp[HW + c];
        if (FB && threadIdx.x < 64) prefetch_aa(p, g, pf);
    }
    if (p.nmaps == 1) pf.wall = p.map_wall[c];   // else the game's map is known only with genv
    else pf.map = p.genv[(size_t)g * MRTS_GENV_WORDS + MRTS_G_MAP];
}
template <int NT>
__device__ __forceinline__ void commit_game(const EngineParams& p, const Lds& L, const StatePf& pf) {
    if (threadIdx.x < MRTS_GENV_WORDS) L.sc[threadIdx.x] = pf.genv;
    const int HW = p.HW;
    if ((int)threadIdx.x < HW) {
        const int c = threadIdx.x;
        L.unit[c] = (uint32_t)pf.cell.x;
        L.uid[c] = pf.cell.y;
        L.act[c] = (uint32_t)pf.cell.z;
        L.seq[c] = (uint32_t)pf.cell.w;
        L.wall[c] = p.nmaps == 1 ? (uint8_t)pf.wall : p.map_wall[(size_t)pf.map * HW + c];
        L.resv[c] = -1;   // reservation holders (step 1)
    }
    __syncthreads();
}

// One game per workgroup (a persistent variant looping over games measured
// slower: hipcc allocates 164 VGPRs for the looped body).
// FB (bot fusion, p.fuse_bots): in a bot game's workgroup, wave 0 decides the
// NEXT tick's bot actions (bots::bot_game on the state just stored) while waves
// 1.. stream this tick's outputs; its LDS follows the step's (launch_all).
template <int NT, int P, typename OT, bool FB>
__device__ __forceinline__ void step_game(const EngineParams& p, const int g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int HW = p.HW;
    const bool early_layout = FB && P == 29 && p.early_bot;
    Lds L = carve(smem, HW, p.W, NT, !FB, FB ? smem + fb_wall_offset(HW, p.W, NT, early_layout) : nullptr);
    const bool botg = FB && g >= p.nsp_games && NT > 64;   // the workgroup runs the next tick's bot
    if (botg) {   // the output words outside the bot's region (fb_outw_offset)
        uint32_t* const region = reinterpret_cast<uint32_t*>(smem + fb_outw_offset(HW, p.W, NT));
        L.outw = early_layout ? reinterpret_cast<uint32_t*>(L.uid) : region;
        L.outm = early_layout ? region : region + HW;
    }
    int* const early_cnt = reinterpret_cast<int*>(smem + fb_early_cnt_offset(HW, p.W, NT, early_layout));
    if (FB && threadIdx.x == 0) *early_cnt = 0;   // read after several barriers below
    // issue priority: the game logic (latency-bound chains of LDS steps and
    // barriers) over other workgroups' output streams (memory-bound), which
    // drop to 0 in emit_outputs' phase B
    __builtin_amdgcn_s_setprio(2);
#ifdef MRTS_STAMPS
    if (threadIdx.x == 0) {   // rows by workgroup (no atomics: they would skew the start stamps);
        // maps of more than 256 cells launch apart from the others (mrts_step_group plans)
        // (no row counter: an atomic on one address by every workgroup sits in the vmcnt
        // queue ahead of the state loads and skewed the first round by ~10 us)
        mrts_stamp_row = (int)blockIdx.x + (HW > 256 ? MRTS_STAMP_ROWS / 2 : 0);
        if (mrts_stamp_row < MRTS_STAMP_ROWS) {
            g_stamp[mrts_stamp_row][0] = (unsigned long long)g | ((unsigned long long)HW << 32);
            g_stamp[mrts_stamp_row][1] = (unsigned long long)(g >= p.nsp_games) | ((unsigned long long)(FB && NT > 64) << 1) |
                                         ((unsigned long long)p.early_bot << 2);
        }
    }
    __syncthreads();
#endif
    MRTS_STAMP(2, threadIdx.x == 0);
    const Grid gd{p.W, p.H, HW};
    const bool pf_ok = HW <= NT;   // state, genv and source rows in one round trip
    const bool pf_wide = !pf_ok && HW <= 4 * NT;   // the same for up to four cells per lane
    StatePf pf;
    WidePf wpf;
    if (game_parked(p, g)) return;   // no tick: its outputs stay zero (mrts_park_games)
    if (pf_ok) prefetch_game<NT, FB>(p, g, pf);
    else if (pf_wide) prefetch_wide<NT>(p, game_of(p, g), g, wpf);
    MRTS_STAMP(15, threadIdx.x == 0);
    if (FB && P == 29 && p.early_bot && g >= p.nsp_games && NT > 64) {   // the early bot's tail arrays start zeroed
        uint32_t* t = reinterpret_cast<uint32_t*>(smem + fb_tail_offset(HW, p.W, NT, true));
        for (int i = threadIdx.x; i < (int)(bots::bot_tail_bytes(HW, p.W) / 4); i += NT) t[i] = 0;
    }
    const Game G = game_of(p, g);
    // Barriers: each phase below is ordered after the last one that wrote what it
    // reads from OTHER lanes; a phase that reads only its own lane's cells (the
    // same c = threadIdx.x + k * NT walk) follows its predecessor without one.
    // Everything zeroed or initialised here is first read after commit_game's barrier.
    if (threadIdx.x < SC_WORDS) L.sc[threadIdx.x] = 0;
    const int posw = (HW + 2 * p.W) / 32 + 1;   // position words (targets as x + y * W + W)
    for (int i = threadIdx.x; i < 2 * posw; i += NT) L.claim[i] = 0;
    // the source-unit rows of this lane's first cell, fetched in the same round
    // trip as the game state (the decode below needs both)
    int src_pre[2] = {0, 0};
    if (pf_ok) {
        src_pre[0] = pf.src0;
        src_pre[1] = pf.src1;
    } else if (!pf_wide && (int)threadIdx.x < HW) {
        for (int v = 0; v < G.nviews; v++) src_pre[v] = p.src[(size_t)(G.env0 + v) * HW + threadIdx.x];
    }
    if (pf_ok) {
        commit_game<NT>(p, L, pf);
    } else if (pf_wide) {
        commit_wide<NT>(p, L, wpf);
    } else {
        for (int c = threadIdx.x; c < HW; c += NT) L.resv[c] = -1;
        load_game<NT>(p, L, g);
    }
    MRTS_STAMP(3, threadIdx.x == 0);
    const int time = L.sc[SC_TIME];
    const int steps0 = L.sc[SC_STEPS], map_now = L.sc[SC_MAP];   // read before any lane can rewrite them (auto-reset)
    // bot-vs-bot game (MicroRTSBotVecEnv): player 0's PlayerAction comes from k_bot too
    const bool bot0 = !G.selfplay && p.bot_ai0 && p.bot_ai0[g - p.nsp_games] >= 0;

    // (1) decode the rows of every idle unit whose cell is in source_unit_mask
    //     (vec_env.py:972-974) + Unit.canExecuteAction, lane-parallel.
    // + pending move/produce reservations (ResourceUsage of unitActions) and whether
    //   a pending produce is over its owner's budget; + the target positions the
    //   agent's move / produce rows claim (step 2a)
    int units = 0;   // player 0's units + player 1's << 16 (SC_HAS)
    // per cell: unit counts, pending reservations / produce budgets; returns the
    // view whose agent row the cell's idle unit may take (-1: none)
    auto cell_pass = [&](int c, uint32_t u) {
        const int ow = u_owner(u);
        if (u != 0 && (ow == 0 || ow == 1)) units += ow ? 1 << 16 : 1;
        const uint32_t pa = L.act[c];
        if (pa) {
            const int code = act_code(pa), ty = code_type(code);
            if (ty == A_MOVE || ty == A_PRODUCE) {
                const int n = nb_cell(gd, c, code_param(code));
                if (n >= 0) L.resv[n] = c;
                if (ty == A_PRODUCE) {
                    const int cost = ut_cost(code_utype(code));
                    if (cost > res_of(L, u_owner(u))) L.sc[SC_OVER] = 1;
                    if (ow == 0 || ow == 1) atomicMax(&L.sc[SC_PMAX + ow], cost);
                    L.prod[atomicAdd(&L.sc[SC_NPEND], 1)] = c;   // (any order: issue() picks candidates by sequence)
                }
            }
        }
        return (u != 0 && ow >= 0 && pa == 0) ? (G.selfplay ? ow : (ow == 0 && !bot0 ? 0 : -1)) : -1;
    };
    // the agent's action row of cell c's idle unit (view v, owner ow): decode +
    // legality + the target claims; returns its aux word
    auto decode_row = [&](int c, int v, int ow) -> uint32_t {
        const int64_t* ra = p.actions + ((size_t)(G.env0 + v) * HW + c) * 7;
        int64_t r[7];   // all 7 components in one round trip
#pragma unroll
        for (int k = 0; k < 7; k++) r[k] = ra[k];
        int64_t ty = r[0];
        int code = -1;
        if (ty == A_NONE) code = code_make(A_NONE, 1, 0);   // NONE(1): param = duration
        else if (ty >= A_MOVE && ty <= A_RETURN) {
            int64_t d = r[ty];
            if (d >= 0 && d < 4) code = code_make((int)ty, (int)d, 0);
        } else if (ty == A_PRODUCE) {
            int64_t d = r[4], t2 = r[5];
            if (d >= 0 && d < 4 && t2 >= 0 && t2 < MRTS_NTYPES) code = code_make(A_PRODUCE, (int)d, (int)t2);
        } else if (ty == A_ATTACK) {
            int64_t a = r[6];
            if (a >= 0 && a < MRTS_ATTACK_GRID * MRTS_ATTACK_GRID) code = code_make(A_ATTACK, (int)a, 0);
        }
        if (code < 0) return 0u;
        const bool lg = legal_code(gd, c, code, L.unit, L.wall, res_of(L, ow));
        claim_target(L, gd, c, code, posw);
        if (code_type(code) == A_PRODUCE) atomicAdd(&L.sc[SC_PSUM + ow], ut_cost(code_utype(code)));
        return CAND | (lg ? LEGAL : 0u) | (uint32_t)code;
    };
    if (!pf_wide) {   // one cell per lane (maps of <= NT cells) or the unprefetched path
        for (int c = threadIdx.x; c < HW; c += NT) {
            const uint32_t u = L.unit[c];
            const int v = cell_pass(c, u);
            uint32_t nw = 0;
            if (v >= 0 && (c == (int)threadIdx.x ? src_pre[v] : p.src[(size_t)(G.env0 + v) * HW + c])) nw = decode_row(c, v, u_owner(u));
            L.aux[c] = nw;
        }
    } else {
        // wider maps: the rows to decode are gathered per wave first (ballots; the
        // source words came with the prefetch, in aux) and then loaded one per lane,
        // so the lane's two to four cells cost one action-row round trip, not one each.
        // The wave's list lives in the ready-set snapshots' array (4 HW words, first used
        // by the cycle): wave w takes [w K 64, (w + 1) K 64), K = cells per lane <= 4.
        const int K = (HW + NT - 1) / NT, lane = threadIdx.x & 63;
        int32_t* const wl = reinterpret_cast<int32_t*>(L.snap) + (threadIdx.x >> 6) * K * 64;
        int wn = 0;
        for (int k = 0; k < K; k++) {   // uniform trip count: every lane takes part in each ballot
            const int c = (int)threadIdx.x + k * NT;
            int e = -1;
            if (c < HW) {
                const uint32_t u = L.unit[c];
                const int v = cell_pass(c, u);
                if (v >= 0 && ((L.aux[c] >> v) & 1u)) e = c | (v << 16);
                L.aux[c] = 0;
            }
            const unsigned long long m = __ballot(e >= 0);
            if (e >= 0) wl[wn + __popcll(m & ((1ull << lane) - 1ull))] = e;
            wn += __popcll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        for (int j = lane; j < wn; j += 64) {
            const int e = wl[j], c = e & 0xFFFF, v = e >> 16;
            L.aux[c] = decode_row(c, v, u_owner(L.unit[c]));
        }
    }
    if (units) atomicAdd(&L.sc[SC_HAS], units);
    // the device bot's PlayerAction for player 1 (k_bot, computed on the state
    // before this tick's issues: JNIGridnetClient.gameStep order)
    const int npa = (!G.selfplay && p.botpa) ? L.sc[SC_NPA] : 0;
    const int npa0 = bot0 ? L.sc[MRTS_G_NPA0] : 0;
    if (npa | npa0) __syncthreads();   // the bot rows' aux words after the decode's (which zeroed them)
    // entry k of player q's PlayerAction: lane k's prefetched word (maps with HW <= NT),
    // else a load; its position in the PlayerAction (the LinkedHashMap rank) rides in aux
    for (int q = 0; q < 2; q++) {
        const int nq = q ? npa : npa0;
        for (int k = threadIdx.x; k < nq; k += NT) {
            const int e = (pf_ok && k == (int)threadIdx.x)     ? (q ? pf.bpa1 : pf.bpa0)
                          : (pf_wide && k == (int)threadIdx.x) ? (q ? wpf.bpa1 : wpf.bpa0)
                                                           : p.botpa[((size_t)(g - p.nsp_games) * 2 + q) * HW + k];
            const int c = e & 0xFFFF, code = e >> 16;
            (q ? L.blist : L.blist0)[k] = c;
            L.aux[c] = CAND | (legal_code(gd, c, code, L.unit, L.wall, res_of(L, q)) ? LEGAL : 0u) | ((uint32_t)k << 12) |
                       (uint32_t)code;
            claim_target(L, gd, c, code, posw);
            if (code_type(code) == A_PRODUCE) atomicAdd(&L.sc[SC_PSUM + q], ut_cost(code_utype(code)));
        }
    }
    // the pending produces (L.prod) were appended in the decode: issue() visits its
    // candidates by sequence word, so their order is free and no ordered compaction is
    // needed; this barrier orders the reservations, claims, SC_OVER / SC_PSUM / SC_PMAX,
    // L.prod and the bot rows before everything below
    __syncthreads();
    const int nprod = L.sc[SC_NPEND];
    // (2a) rows that interact with nothing else this tick issue lane-parallel: a
    //      row (agent or device bot) whose target position, if a move or produce,
    //      no other row (either player) and no pending assignment claims, while no
    //      pending produce is over its owner's budget (which would make every new
    //      action inconsistent); a produce besides only while all of its player's
    //      produce rows this tick together with the player's dearest pending
    //      produce fit the player's resources (SC_PSUM + SC_PMAX): then no prefix of
    //      the PlayerAction's ResourceUsage exceeds them (fromVectorAction keeps it
    //      and every later row) and no pair of produces is over budget (issue()
    //      finds no candidate for it, nor does any later row find it).  Such a row
    //      meets no candidate in issue() and no other row in fromVectorAction's
    //      filter, and no ordered row of either player meets it, so issuing it out
    //      of order is exact: its LinkedHashMap rank is still its cell (agent rows)
    //      or its position in the bot's PlayerAction.  (A parallel produce is never
    //      a candidate of an ordered row, so it stays out of L.prod.)  Everything
    //      else takes the ordered path (2b).
    const bool over = L.sc[SC_OVER] != 0;
    {
        if (!over) {
            int left = 0;   // this lane's rows left to (2b)
            for (int c = threadIdx.x; c < HW; c += NT) {
                const uint32_t nw = L.aux[c];
                if (!(nw & CAND)) continue;
                const uint32_t u = L.unit[c];
                const int q = u_owner(u);
                const bool botrow = !G.selfplay && (q != 0 || bot0);
                const int rank = botrow ? (int)((nw >> 12) & 0xFFFu) : c;
                const int code = (int)(nw & 0xFFFu), ty = code_type(code);
                if (ty == A_PRODUCE && L.sc[SC_PSUM + q] + L.sc[SC_PMAX + q] > res_of(L, q)) { left++; continue; }
                int n = -1;
                if (ty == A_MOVE || ty == A_PRODUCE) {
                    const int b = unchecked_pos(gd, c, code_param(code)) + p.W;
                    n = nb_cell(gd, c, code_param(code));
                    if (((L.claim[posw + (b >> 5)] >> (b & 31)) & 1u) || (n >= 0 && L.resv[n] >= 0)) { left++; continue; }
                }
                int cur = code, dur = 0;
                if (ty == A_NONE) dur = code_param(code);
                else if (!(nw & LEGAL)) { dur = eta_code(code, u_type(u)); cur = code_make(A_NONE, 0, 0); }
                const int ct = code_type(cur);
                L.act[c] = act_make(cur, ct == A_NONE ? time + dur : time + eta_code(cur, u_type(u)));
                L.seq[c] = seq_make(time, q, rank);
                if (ct == A_MOVE || ct == A_PRODUCE) L.resv[n] = c;
                if (ct == A_HARVEST || ct == A_RETURN) atomicAdd(&L.sc[SC_R0 + 6 * q + 1], 1);
                if (ct == A_ATTACK) atomicAdd(&L.sc[SC_R0 + 6 * q + 4], 1);
                if (ct == A_PRODUCE) {   // ai.reward.ProduceWorker / ProduceBuilding / ProduceCombatUnit
                    const int pu = code_utype(cur);
                    atomicAdd(&L.sc[SC_R0 + 6 * q + (pu == WORKER ? 2 : (pu == BASE || pu == BARRACKS) ? 3 : 5)], 1);
                }
                L.aux[c] = nw & ~CAND;   // issued
            }
            if (left) atomicAdd(&L.sc[SC_NLEFT], left);
        }
    }
    // (2b) the ordered path for the rest: listed (an ordered compaction, the ranks of
    // agent rows being their cells) only when (2a) left any row -- most ticks it
    // leaves none.  The barrier orders (2a)'s issues before the ordered part.
    __syncthreads();
    int nrows = 0;
    if (over || L.sc[SC_NLEFT]) nrows = compact_cells<NT>(HW, [&](int c) { return (L.aux[c] & CAND) != 0; }, L.list, L.ballot);
    MRTS_STAMP(4, threadIdx.x == 0);
    // (2) ordered part: p0 then p1 (bot envs: the passive bot issues only NONEs)
    if (threadIdx.x == 0) {
        L.sc[SC_NPROD] = nprod;
        if (bot0) issue_player(p, L, gd, 0, L.blist0, npa0, false);
        else issue_player(p, L, gd, 0, L.list, nrows, true);
        if (G.selfplay) issue_player(p, L, gd, 1, L.list, nrows, true);
        else if (npa > 0) issue_player(p, L, gd, 1, L.blist, npa, false);
    }
    __syncthreads();
    MRTS_STAMP(5, threadIdx.x == 0);
    // (3) fillWithNones(gs, player, 1) for every idle unit (both players); the
    //     cycle's first passes below read each cell on the lane that wrote it.
    //     claim[0, posw) (dead since the decode's claims) is cleared for the ready
    //     set's harvest-pile check.
    for (int i = threadIdx.x; i < posw; i += NT) L.claim[i] = 0;
    for (int c = threadIdx.x; c < HW; c += NT) {
        uint32_t u = L.unit[c];
        if (u != 0 && u_owner(u) >= 0 && L.act[c] == 0) {
            L.act[c] = act_make(A_NONE, time + 1);
            L.seq[c] = seq_make(time, u_owner(u), 4095);
        }
    }
    // (4) GameState.cycle(): time++, execute ready assignments in issue order
    const int now = time + 1;
    for (int c = threadIdx.x; c < HW; c += NT) {
        uint32_t a = L.act[c];
        if (a && act_done(a) <= now && code_type(act_code(a)) == A_NONE) L.act[c] = 0;
    }
    // the ready cells in L.list, their sequence words in L.aux (dead since the issue),
    // appended in any order: they are ranked by sequence word below
    for (int c = threadIdx.x; c < HW; c += NT) {
        const uint32_t a = L.act[c];
        if (a != 0 && act_done(a) <= now) {
            const int pos = atomicAdd(&L.sc[SC_NREADY], 1);
            L.list[pos] = c;
            L.aux[pos] = L.seq[c];
        }
    }
    __syncthreads();
    const int nready = L.sc[SC_NREADY];
    // snapshots of the ready assignments in LinkedHashMap (issue-sequence)
    // order: lane-parallel rank by sequence word (unique among non-NONE actions);
    // in the same pass, unitActions.remove and whether the set commutes:
    // independent ready sets (no attack, no two harvests of one pile) do -- every
    // target cell is distinct (moves / produces hold reservations), resources only
    // add up, and produced units take ids in issue order.  (Attacks on cells no
    // other ready action touches would commute too; run in parallel that way they
    // measured neutral at 1024 and slower at 8192 envs: DESIGN.md §5.)
    int serial = 0, nprodr = 0;
    for (int i = threadIdx.x; i < nready; i += NT) {
        const int c = L.list[i];
        const uint32_t sq = L.aux[i];
        int rank = 0, j = 0;
        for (; j + 4 <= nready; j += 4) {   // four sequence words per LDS read, no pointer chase
            const uint4 v = *reinterpret_cast<const uint4*>(L.aux + j);
            rank += (v.x < sq) + (v.y < sq) + (v.z < sq) + (v.w < sq);
        }
        for (; j < nready; j++) rank += L.aux[j] < sq;
        const int code = act_code(L.act[c]), ty = code_type(code);
        L.snap[rank] = make_int4(c, (int)L.unit[c], code, L.uid[c]);
        L.act[c] = 0;   // unitActions.remove (each ready cell is read by its own lane only)
        if (ty == A_ATTACK) serial = 1;
        nprodr += ty == A_PRODUCE;
        if (ty == A_HARVEST) {
            const int n = nb_cell(gd, c, code_param(code));
            if (n >= 0 && (atomicOr(&L.claim[n >> 5], 1u << (n & 31)) >> (n & 31)) & 1u) serial = 1;
        }
    }
    if (nprodr) atomicAdd(&L.sc[SC_RPROD], nprodr);   // the ids the produced units take (SC_RPROD starts at 0)
    const int uid0 = L.sc[SC_UID];   // read before lane 0 may advance it (below)
    // (the OR over lanes through an LDS word: __syncthreads_or's static LDS would cost
    // every workgroup 256 B)
    if (serial) L.sc[SC_SERIAL] = 1;
    __syncthreads();
    serial = L.sc[SC_SERIAL];
    MRTS_STAMP(6, threadIdx.x == 0);
    if (serial) {
        if (threadIdx.x == 0)
            for (int i = 0; i < nready; i++) execute_one(L, gd, L.snap[i]);
    } else {
        for (int i = threadIdx.x; i < nready; i += NT) {
            const int4 sn = L.snap[i];
            int puid = -1;
            if (code_type(sn.z) == A_PRODUCE) {
                puid = uid0;
                for (int j = 0; j < i; j++) puid += code_type(L.snap[j].z) == A_PRODUCE;
            }
            execute_one<true>(L, gd, sn, puid);
        }
    }
    // (no barrier: the scalars below are lane 0's, SC_UID is no longer read, and the
    // unit counts -- kept by execute_one -- are read behind the next barrier)
    if (threadIdx.x == 0) {
        L.sc[SC_TIME] = now;
        L.sc[SC_TICKS]++;
        L.sc[MRTS_G_SERIAL] += serial;      // rollout statistics (mrts_game_stats)
        L.sc[MRTS_G_ORDERED] += nrows;
        if (now >= MRTS_MAX_TIME) atomicOr(&L.sc[SC_ERR], MRTS_ERR_TIME_OVERFLOW);   // the executing lanes may be ORing too
        if (!serial)
            L.sc[SC_UID] += L.sc[SC_RPROD];
    }
    __syncthreads();
    // (5) PhysicalGameState.gameover / winner: the unit counts of the decode pass,
    //     less the units attacks removed, plus the produced ones (execute_one)
    const int has = L.sc[SC_HAS];
    const bool has0 = (has & 0xFFFF) != 0, has1 = (has >> 16) != 0;
    const bool gameover = !(has0 && has1);
    const int winner = (has0 && !has1) ? 0 : (has1 && !has0) ? 1 : -1;
    // (6) rewards / done (JNIGridnetVecClient.gameStep terminal handling)
    const int steps = steps0 + 1;
    const bool reset = gameover || steps >= p.max_steps;
    if (threadIdx.x < 6 * G.nviews) {
        int v = threadIdx.x / 6, k = threadIdx.x % 6;
        int env = G.env0 + v;
        double r = k == 0 ? (gameover ? (winner == v ? 1.0 : -1.0) : 0.0) : (double)L.sc[SC_R0 + 6 * v + k];
        p.raw_reward[(size_t)env * 6 + k] = r;
        p.done[(size_t)env * 6 + k] = (uint8_t)((gameover || (k == 0 && reset)) ? 1 : 0);
    }
    if (p.reward && threadIdx.x < G.nviews) {   // fused `reward @ reward_weight`, done[:, 0]
        const int v = threadIdx.x, env = G.env0 + v;
        double s = 0.0;
        for (int k = 0; k < 6; k++) {
            double r = k == 0 ? (gameover ? (winner == v ? 1.0 : -1.0) : 0.0) : (p.shaping ? (double)L.sc[SC_R0 + 6 * v + k] : 0.0);
            s = __dadd_rn(s, __dmul_rn(r, p.rw[k]));   // no FMA contraction: numpy's sequential dot
        }
        p.reward[env] = s;
        p.done0[env] = (uint8_t)(reset ? 1 : 0);
    }
    // (no barrier: the rewards read only SC_R0.. words, which the reset leaves
    // alone, and nothing above reads the cell arrays it rewrites)
    if (reset) {
        reset_into_lds<NT>(p, L, map_now);
        if (threadIdx.x == 0) {
            L.sc[SC_AA_N] = L.sc[MRTS_G_AA_N0] = 0;   // ai1 / ai2.reset()
            L.sc[MRTS_G_EPISODES]++;
        }
    } else if (threadIdx.x == 0) {
        L.sc[SC_STEPS] = steps;
    }
    __syncthreads();
    // (7) write back + one-hot observation of every view
    MRTS_STAMP(7, threadIdx.x == 0);
    store_game<NT>(p, L, g);
    const int res0 = L.sc[SC_RES0], res1 = L.sc[SC_RES1];   // before the early bot may reuse the scalars' bytes
    // + getMasks of the next tick (bound mask outputs): every read of this
    //   game's source rows (phase 1) is behind the barriers above
    // Early bot (P == 29, p.early_bot: full observability, and for this size the bot
    // writes none of the arrays phase A reads -- unit / act / wall stay as stored, the
    // step's scalars and visibility words are left alone, its small arrays go to the
    // tail region): once store_game has read the arrays the bot reuses, the workgroup
    // builds the bot's setup, then wave 0 starts the next tick's bot at once while
    // waves 1.. build the output words and stream them, meeting at an LDS counter
    // instead of a workgroup barrier.  Otherwise wave 0 helps with phase A and starts
    // the bot behind its barrier (the step's arrays are dead by then: only L.outw is
    // read on).  One bot_game call site for both: the inlined bot is most of this
    // kernel's code.
    const bool early = early_layout && botg;
    unsigned char* const tail = smem + fb_tail_offset(HW, p.W, NT, early_layout);
    if (early) {
        __syncthreads();
        bot_setup_workgroup<NT>(p, smem, tail, L.wall);
        __syncthreads();
        MRTS_STAMP(14, threadIdx.x == 0);
    }
    if (!early || threadIdx.x >= 64)
        emit_outputs<NT, P, OT>(p, L, G, true, p.mask != nullptr, res0, res1, botg ? 64 : 0, early ? early_cnt : nullptr);
    if (FB && botg && threadIdx.x < 64) {
        if (early) __builtin_amdgcn_s_setprio(3);   // the latency-bound bot wave first; the streaming waves are memory-bound
        bots::bot_game<true>(p, g - p.nsp_games, 1, smem, L.sc, pf_ok, pf.aa, pf.aa2, tail, L.wall, early);
        MRTS_STAMP(13, threadIdx.x == 0);
    }
}

// One step launch over the games of one or more engines (map-size buckets of one
// batch, mrts_step_group): the grid is cut into segments of consecutive games of
// one engine; a workgroup finds its segment with a scalar scan of the table (at
// most 2 * MRTS_STEP_GROUP_MAX entries) and runs that engine's game.  Each
// engine's arrays, map size and LDS carve are its own; the launch's dynamic LDS
// is the largest member's.  A single engine is a one-member, one-segment group.
template <int NT, int P, typename OT, bool FB = false>
__global__ __launch_bounds__(NT) void k_step(const StepGroup sg) {
    const int b = blockIdx.x;
    int k = 0;
    while (k + 1 < sg.nseg && b >= sg.seg_block[k + 1]) k++;
    step_game<NT, P, OT, FB>(sg.e[sg.seg_member[k]], sg.seg_game[k] + (b - sg.seg_block[k]));
}

// ---------------------------------------------------------------------------
// render("rgb_array") (vec_env.py:1075-1084): a size x size RGB frame of one
// game, one lane per pixel.  The Java PhysicalGameStatePanel is absent, so the
// drawing rules are this engine's own (restated pixel for pixel
// by oracle_py.render_frame): cells of cs = size / max(W, H) pixels centred in
// the frame, grid lines, walls, buildings / resources as inset squares, mobile
// units as discs, an owner-coloured rim (player 0 blue, player 1 red) and a
// hit-point bar on damaged units.
__device__ __forceinline__ uint32_t render_type_rgb(int t) {
    switch (t) {
    case RESOURCE: return 0x00A000u;
    case BASE: return 0xFFFFFFu;
    case BARRACKS: return 0xA0A0A0u;
    case WORKER: return 0x808080u;
    case LIGHT: return 0xFF8000u;
    case HEAVY: return 0xFFFF00u;
    default: return 0x00FFFFu;   // RANGED
    }
}

__global__ __launch_bounds__(256) void k_render(const int4* __restrict__ cells, const uint8_t* __restrict__ wall, int W, int H,
                                              int size, uint8_t* __restrict__ rgb) {
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= size * size) return;
    const int px = pix % size, py = pix / size;
    const int cs = size / max(W, H), ox = (size - cs * W) / 2, oy = (size - cs * H) / 2;
    uint32_t col = 0;
    const int gx = px - ox, gy = py - oy;
    if (gx >= 0 && gy >= 0 && gx < cs * W && gy < cs * H) {
        const int cx = gx / cs, cy = gy / cs, lx = gx - cx * cs, ly = gy - cy * cs, c = cy * W + cx;
        col = wall[c] ? 0x205020u : 0u;
        if (lx == 0 || ly == 0) col = 0x303030u;
        const uint32_t u = (uint32_t)cells[c].x;
        if (u != 0) {
            const int t = u_type(u), ow = u_owner(u), m = cs / 8, b = max(1, cs / 16);
            const bool building = t == RESOURCE || t == BASE || t == BARRACKS;
            bool inside, rim;
            if (building) {
                inside = lx >= m && ly >= m && lx < cs - m && ly < cs - m;
                rim = lx < m + b || ly < m + b || lx >= cs - m - b || ly >= cs - m - b;
            } else {
                const int r2 = cs * 3 / 4, dx = 2 * lx + 1 - cs, dy = 2 * ly + 1 - cs, d2 = dx * dx + dy * dy;
                inside = d2 <= r2 * r2;
                rim = d2 > (r2 - 2 * b) * (r2 - 2 * b);
            }
            if (inside) {
                col = render_type_rgb(t);
                if (rim && ow >= 0) col = ow == 0 ? 0x0000FFu : 0xFF0000u;
            }
            const int hp = u_hp(u), mhp = ut_hp(t);
            if (t != RESOURCE && hp < mhp && ly >= cs - m - 2 * b && ly < cs - m && lx >= m && lx < m + (cs - 2 * m) * hp / mhp)
                col = 0xFF0000u;
        }
    }
    rgb[3 * (size_t)pix] = (uint8_t)(col >> 16);
    rgb[3 * (size_t)pix + 1] = (uint8_t)(col >> 8);
    rgb[3 * (size_t)pix + 2] = (uint8_t)col;
}

// ---------------------------------------------------------------------------
// Counter-based masked sampler (hello_world.py:27-64 semantics), Philox4x32-10
// keyed (seed) with counter (cell, env, step, half) -- identical stream to the
// oracle's ovec_sample_actions.  `env` is the GLOBAL env index (env0 + local
// row), so a shard of envs [env0, env0 + n) draws exactly the actions of that
// slice of one larger run (multi-GPU sharding).
// (each round's two 32x32 products as 64-bit ones: one v_mad_u64_u32 each instead of
// a v_mul_hi_u32 + v_mul_lo_u32 pair, both quarter rate; the sampler's bound is its
// memory round trips, not these multiplies: one block per row measured 32.5 -> 32.0 us,
// profiles/r04_ab/r04u)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// One row (env e, cell c): the 78 mask channels as bits lo (0..63) | hi (64..77);
// per component k, a uniform pick among the valid entries (uniform over all
// entries when none is valid), from two Philox4x32-10 blocks of counter
// (c, e, step, 0|1) -- the oracle's ovec_sample_actions stream.
// The row's eight random words: they depend on (cell, env, step, seed) only, so a
// caller can draw them while the row's mask bits are still in flight.
__device__ __forceinline__ void philox_row(int e, int c, uint64_t seed, uint32_t step, uint32_t r[8]) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        uint32_t ctr[4] = {(uint32_t)c, (uint32_t)e, step, (uint32_t)h};
        philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        r[4 * h] = ctr[0]; r[4 * h + 1] = ctr[1]; r[4 * h + 2] = ctr[2]; r[4 * h + 3] = ctr[3];
    }
}
__device__ __forceinline__ void select_row(uint64_t lo, uint64_t hi, const uint32_t r[8], int64_t* out) {
    const int off[7] = {0, 6, 10, 14, 18, 22, 29};
    const int len[7] = {6, 4, 4, 4, 4, 7, 49};
#pragma unroll
    for (int k = 0; k < 7; k++) {
        uint64_t seg = (lo >> off[k]) | (off[k] ? (hi << (64 - off[k])) : 0);   // bits [off, off+len)
        seg &= (1ull << len[k]) - 1ull;
        const int nvalid = __popcll(seg);
        int pick;
        if (nvalid == 0) {
            pick = (int)(((uint64_t)r[k] * (uint32_t)len[k]) >> 32);
        } else {
            int t = (int)(((uint64_t)r[k] * (uint32_t)nvalid) >> 32);
            for (; t > 0; t--) seg &= seg - 1ull;   // drop the t lowest set bits
            pick = __builtin_ctzll(seg);
        }
        out[k] = pick;
    }
}
__device__ __forceinline__ void sample_row(uint64_t lo, uint64_t hi, int e, int c, uint64_t seed, uint32_t step, int64_t* out) {
    uint32_t r[8];
    philox_row(e, c, seed, step, r);
    select_row(lo, hi, r, out);
}

// Persistent, software-pipelined: every WAVE owns groups of SW = 32 consecutive
// (env, cell) rows (32 x 312 B of int32 mask, contiguous).  While a group is
// folded into 78-bit words in the wave's LDS slice and sampled (one lane per
// row), the NEXT group's 10 dwordx4 loads per lane are already in flight in a
// second register buffer, so the HBM stream never idles behind the Philox /
// selection arithmetic.  The 7 int64 components per row are staged in LDS and
// written back with coalesced 16-byte stores.  No block barriers: a wave's own
// LDS operations complete in order.
constexpr int SW = 32;                                   // rows per group (one wave)
constexpr int SWAVES = 4;                                // waves per workgroup
constexpr int SNV = (SW * MRTS_MASK_CH / 4 + 63) / 64;   // dwordx4 loads per lane per group (10)


struct SampleBuf {
    int4 v[SNV];
};

__device__ __forceinline__ void sample_load(SampleBuf& B, const int32_t* __restrict__ mask, long long grp, long long rows) {
    const long long row0 = grp * SW;
    const int rb = (int)min((long long)SW, rows - row0);
    const int nv = rb * MRTS_MASK_CH / 4;
    const int4* m4 = reinterpret_cast<const int4*>(mask + row0 * MRTS_MASK_CH);
    // Unconditional loads (tail lanes re-read the group's last int4 and are
    // masked when consumed): no branch around a load, so hipcc can count them and
    // wait with vmcnt(SNV) for this group while the next one stays in flight.
#pragma unroll
    for (int j = 0; j < SNV; j++) {
        const int k = min(j * 64 + (int)(threadIdx.x & 63), nv - 1);
        const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(m4 + k));   // streamed once
        B.v[j] = make_int4(t.x, t.y, t.z, t.w);
    }
}

__device__ __forceinline__ void sample_group(const SampleBuf& B, const int32_t* __restrict__ mask, long long grp, long long rows,
                                             int hw, int env0, uint64_t seed, uint32_t step, int64_t* __restrict__ act,
                                             uint32_t* s_bits, int64_t* s_out) {
    const int lane = threadIdx.x & 63;
    const long long row0 = grp * SW;
    const int rb = (int)min((long long)SW, rows - row0);
    const int nel = rb * MRTS_MASK_CH, nv = nel >> 2;
    for (int i = lane; i < SW * 3; i += 64) s_bits[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int j = 0; j < SNV; j++) {
        const int k = j * 64 + lane;
        const int4 v = B.v[j];
        if (k >= nv || (v.x | v.y | v.z | v.w) == 0) continue;   // most cells hold no idle unit
        int e = 4 * k;
        int r = e / MRTS_MASK_CH, ch = e - r * MRTS_MASK_CH;
        const int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (vv[q]) atomicOr(&s_bits[3 * r + (ch >> 5)], 1u << (ch & 31));
            if (++ch == MRTS_MASK_CH) { ch = 0; r++; }
        }
    }
    for (int e = 4 * nv + lane; e < nel; e += 64) {   // odd row count: the last 2 int32
        if (mask[row0 * MRTS_MASK_CH + e]) {
            int r = e / MRTS_MASK_CH, ch = e - r * MRTS_MASK_CH;
            atomicOr(&s_bits[3 * r + (ch >> 5)], 1u << (ch & 31));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < rb) {
        const long long idx = row0 + lane;
        const int e = (int)(idx / hw), c = (int)(idx - (long long)e * hw);
        const uint64_t lo = (uint64_t)s_bits[3 * lane] | ((uint64_t)s_bits[3 * lane + 1] << 32);
        const uint64_t hi = s_bits[3 * lane + 2];
        sample_row(lo, hi, env0 + e, c, seed, step, s_out + lane * 7);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    int64_t* ob = act + row0 * 7;   // 16-B aligned: SW * 56 B per group
    const int onel = rb * 7, onv = onel >> 1;
    int4* o4 = reinterpret_cast<int4*>(ob);
    const int4* s4 = reinterpret_cast<const int4*>(s_out);
    for (int k = lane; k < onv; k += 64) o4[k] = s4[k];
    if ((onel & 1) && lane == 0) ob[onel - 1] = s_out[onel - 1];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

constexpr int SAMPLE_BLOCKS_PER_CU = 16;   // measured best (round 1: 2 -> 151 us, 4 -> 138, 8 -> 133, 16 -> 127, 64 -> 178)
__global__ __launch_bounds__(64 * SWAVES) void k_sample(const int32_t* __restrict__ mask, int n, int hw, int env0,
                                                        uint64_t seed, uint32_t step, int64_t* __restrict__ act) {
    __shared__ uint32_t s_bits[SWAVES][SW * 3];
    __shared__ __attribute__((aligned(16))) int64_t s_out[SWAVES][SW * 7];
    const int w = threadIdx.x >> 6;
    const long long rows = (long long)n * hw;
    const long long ngrp = (rows + SW - 1) / SW;
    const long long stride = (long long)gridDim.x * SWAVES;
    long long grp = (long long)blockIdx.x * SWAVES + w;
    if (grp >= ngrp) return;
    SampleBuf A, B;
    sample_load(A, mask, grp, rows);
    while (true) {   // two groups per trip: A is consumed while B loads, then the reverse
        const long long g1 = grp + stride;   // past the end: a harmless re-read of the last group
        sample_load(B, mask, min(g1, ngrp - 1), rows);
        sample_group(A, mask, grp, rows, hw, env0, seed, step, act, s_bits[w], s_out[w]);
        if (g1 >= ngrp) break;
        const long long g2 = g1 + stride;
        sample_load(A, mask, min(g2, ngrp - 1), rows);
        sample_group(B, mask, g1, rows, hw, env0, seed, step, act, s_bits[w], s_out[w]);
        if (g2 >= ngrp) break;
        grp = g2;
    }
}

// Source-guided variant: the same stream and output, given the source channel
// as well.  getMasks sets no channel of a cell whose source bit is 0 (no idle
// unit of the player: UnitAction.getValidActionArray is all zero), so only the
// mask rows of source cells are read -- a few per cent of the 78-channel rows
// on basesWorkers -- while every row's 7 components are still drawn and
// written.  One wave per 64 consecutive rows: the wave reads the rows of its
// active lanes cooperatively (channel k on lane k, two coalesced loads per row,
// up to SRC_ROWS (4) rows in flight) and folds each with two ballots.  Measured
// and refuted in round 5 (profiles/r05_ab/): writing every row's no-valid-entry
// draw first and patching the source rows after (sampler 32.6 -> 35.6 us, and the
// next k_step +8 us); two 64-row groups per wave sharing one chain of round trips
// (32.7 -> 32.4 us, configs[1] 2 % slower).
constexpr int SR_WAVES = 4;
constexpr int SRC_ROWS = 4;   // source rows per round trip (8 and 16 measured slower, profiles/r04_ab/r04v)
// one block's 4 x 64 rows of one batch (k_sample_src: block = blockIdx.x; the grouped
// launch: the block's index inside its segment)
__device__ __forceinline__ void sample_src_block(const int32_t* __restrict__ mask, const int32_t* __restrict__ src, int n, int hw,
                                                 int env0, uint64_t seed, uint32_t step, int64_t* __restrict__ act, long long blk,
                                                 int64_t (*s_out)[64 * 7]) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long rows = (long long)n * hw;
    const long long row0 = (blk * SR_WAVES + w) * 64;
    if (row0 >= rows) return;
    const int rb = (int)min(64ll, rows - row0);
    const bool in = lane < rb;
    // unconditional load (tail lanes re-read the last row): no branch around it, so
    // its wait falls after the row's Philox words, which are drawn while the source
    // word (and then the mask rows) are in flight
    const int s_raw = src[row0 + min(lane, rb - 1)];
    uint32_t r8[8];
    const unsigned idx = (unsigned)(row0 + lane);   // rows = n * hw < 2^31 (mrts_sample_actions_src checks)
    const int e = (int)(idx / (unsigned)hw), c = (int)(idx - (unsigned)e * (unsigned)hw);
    philox_row(env0 + e, c, seed, step, r8);
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("" : "+v"(r8[k]));   // computed here, not sunk to their use after the loads
    const int s = in ? s_raw : 0;
    uint64_t pending = __ballot(s != 0);
    uint64_t lo = 0, hi = 0;   // this lane's row as 78 bits
    while (pending) {          // wave-uniform; SRC_ROWS source rows per round trip
        int r[SRC_ROWS];
#pragma unroll
        for (int k = 0; k < SRC_ROWS; k++) {
            r[k] = pending ? __builtin_ctzll(pending) : r[0];   // repeats r[0]
            pending &= pending - 1ull;
        }
        int v0[SRC_ROWS], v1[SRC_ROWS];
#pragma unroll
        for (int k = 0; k < SRC_ROWS; k++) {   // all the loads in flight before the first ballot
            const int32_t* m = mask + (row0 + r[k]) * MRTS_MASK_CH;   // (a repeated row re-reads the same bits)
            v0[k] = __builtin_nontemporal_load(m + lane);
            v1[k] = __builtin_nontemporal_load(m + 64 + min(lane, MRTS_MASK_CH - 65));
        }
#pragma unroll
        for (int k = 0; k < SRC_ROWS; k++) {
            const uint64_t b0 = __ballot(v0[k] != 0);
            const uint64_t b1 = __ballot(lane < MRTS_MASK_CH - 64 && v1[k] != 0);
            if (lane == r[k]) { lo = b0; hi = b1; }
        }
    }
    if (in) select_row(lo, hi, r8, s_out[w] + lane * 7);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    int64_t* ob = act + row0 * 7;   // 16-B aligned: 64 * 56 B per wave
    const int onel = rb * 7, onv = onel >> 1;
    int4* o4 = reinterpret_cast<int4*>(ob);
    const int4* s4 = reinterpret_cast<const int4*>(s_out[w]);
    for (int k = lane; k < onv; k += 64) {   // non-temporal: k_step reads ~2 % of the rows back
        const int4 t = s4[k];
        const v4i v = {t.x, t.y, t.z, t.w};
        __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(o4 + k));
    }
    if ((onel & 1) && lane == 0) ob[onel - 1] = s_out[w][onel - 1];
}
__global__ __launch_bounds__(64 * SR_WAVES) void k_sample_src(const int32_t* __restrict__ mask, const int32_t* __restrict__ src, int n,
                                                           int hw, int env0, uint64_t seed, uint32_t step,
                                                           int64_t* __restrict__ act) {
    __shared__ __attribute__((aligned(16))) int64_t s_out[SR_WAVES][64 * 7];
    sample_src_block(mask, src, n, hw, env0, seed, step, act, blockIdx.x, s_out);
}
// Several batches (a mixed batch's size buckets) in one launch: segment k owns blocks
// [end[k-1], end[k]); a block finds its segment with a scalar scan of the table.
struct SampleSeg {
    const int32_t* mask;
    const int32_t* src;
    int64_t* act;
    int n, hw, env0;
};
struct SampleGroup {
    SampleSeg seg[MRTS_SAMPLE_GROUP_MAX];
    long long end[MRTS_SAMPLE_GROUP_MAX];
    int nseg;
};
__global__ __launch_bounds__(64 * SR_WAVES) void k_sample_src_group(const SampleGroup g, uint64_t seed, uint32_t step) {
    __shared__ __attribute__((aligned(16))) int64_t s_out[SR_WAVES][64 * 7];
    const long long b = blockIdx.x;
    int k = 0;
    while (k + 1 < g.nseg && b >= g.end[k]) k++;
    const SampleSeg& sg = g.seg[k];
    sample_src_block(sg.mask, sg.src, sg.n, sg.hw, sg.env0, seed, step, sg.act, b - (k ? g.end[k - 1] : 0), s_out);
}

// ---------------------------------------------------------------------------
// launchers


// One engine's step launch.  With both selfplay and bot games, the bot games take
// the first workgroups: workgroups start in grid order, and a bot game's chain (the
// fused bot after the tick) is the longest, so the short selfplay games fill the last
// round (4096 selfplay + 4096 bot envs, 16x16: step 215 -> 196 us,
// profiles/r03_ab/ab20_single_engine_bots_first/).
static StepGroup one_engine(const EngineParams& p) {
    StepGroup sg{};
    sg.e[0] = p;
    if (p.nsp_games > 0 && p.nsp_games < p.G) {
        sg.seg_game[0] = p.nsp_games;
        sg.seg_block[1] = p.G - p.nsp_games;
        sg.seg_game[1] = 0;
        sg.seg_block[2] = p.G;
        sg.nseg = 2;
    } else {
        sg.seg_block[1] = p.G;
        sg.nseg = 1;
    }
    return sg;
}

// the step kernel of a launch's (planes, obs type, bot fusion)
template <int NT>
static void launch_step(const StepGroup& sg, int grid, size_t sh, hipStream_t s, bool partial, bool fl, bool fb) {
    if (fb) {
        if (partial) {
            if (fl) hipLaunchKernelGGL((k_step<NT, 31, float, true>), dim3(grid), dim3(NT), sh, s, sg);
            else hipLaunchKernelGGL((k_step<NT, 31, int32_t, true>), dim3(grid), dim3(NT), sh, s, sg);
        } else {
            if (fl) hipLaunchKernelGGL((k_step<NT, 29, float, true>), dim3(grid), dim3(NT), sh, s, sg);
            else hipLaunchKernelGGL((k_step<NT, 29, int32_t, true>), dim3(grid), dim3(NT), sh, s, sg);
        }
    } else {
        if (partial) {
            if (fl) hipLaunchKernelGGL((k_step<NT, 31, float>), dim3(grid), dim3(NT), sh, s, sg);
            else hipLaunchKernelGGL((k_step<NT, 31, int32_t>), dim3(grid), dim3(NT), sh, s, sg);
        } else {
            if (fl) hipLaunchKernelGGL((k_step<NT, 29, float>), dim3(grid), dim3(NT), sh, s, sg);
            else hipLaunchKernelGGL((k_step<NT, 29, int32_t>), dim3(grid), dim3(NT), sh, s, sg);
        }
    }
}

template <int NT>
static hipError_t launch_all(const EngineParams& p, int kind, hipStream_t s, const int32_t* games, const int32_t* maps, int count) {
    size_t sh = lds_bytes(p.HW, p.W, NT);
    int grid = p.G;
    if (kind == 0) {   // reset
        grid = games ? count : p.G;
        if (grid == 0) return hipSuccess;
        if (p.partial_obs) {
            if (p.obs_float) hipLaunchKernelGGL((k_reset<NT, 31, float>), dim3(grid), dim3(NT), sh, s, p, games, maps, count);
            else hipLaunchKernelGGL((k_reset<NT, 31, int32_t>), dim3(grid), dim3(NT), sh, s, p, games, maps, count);
        } else {
            if (p.obs_float) hipLaunchKernelGGL((k_reset<NT, 29, float>), dim3(grid), dim3(NT), sh, s, p, games, maps, count);
            else hipLaunchKernelGGL((k_reset<NT, 29, int32_t>), dim3(grid), dim3(NT), sh, s, p, games, maps, count);
        }
    } else if (kind == 1) {
        hipLaunchKernelGGL((k_masks<NT>), dim3(grid), dim3(NT), sh, s, p);
    } else if (kind == 3) {
        if (p.partial_obs) {
            if (p.obs_float) hipLaunchKernelGGL((k_outputs<NT, 31, float>), dim3(grid), dim3(NT), sh, s, p);
            else hipLaunchKernelGGL((k_outputs<NT, 31, int32_t>), dim3(grid), dim3(NT), sh, s, p);
        } else {
            if (p.obs_float) hipLaunchKernelGGL((k_outputs<NT, 29, float>), dim3(grid), dim3(NT), sh, s, p);
            else hipLaunchKernelGGL((k_outputs<NT, 29, int32_t>), dim3(grid), dim3(NT), sh, s, p);
        }
    } else {
        const bool fb = p.fuse_bots && NT > 64;
        if (fb) sh = fb_lds_bytes(p.HW, p.W, NT, !p.partial_obs && p.early_bot);
        launch_step<NT>(one_engine(p), grid, sh, s, p.partial_obs, p.obs_float, fb);
    }
    return hipGetLastError();
}

// Workgroup size of a map size: one lane per cell up to 256 lanes; the bot-fused
// step needs a wave besides the bot's, so maps of <= 64 cells take 128 lanes there.
__host__ __device__ inline int step_nt(int HW, bool fused) { return HW <= 64 && !fused ? 64 : HW <= 128 ? 128 : 256; }

static hipError_t dispatch(const EngineParams& p, int kind, hipStream_t s, const int32_t* games, const int32_t* maps, int count) {
    if (kind == 2 && p.fuse_bots) return step_nt(p.HW, true) == 128 ? launch_all<128>(p, kind, s, games, maps, count)
                                                                      : launch_all<256>(p, kind, s, games, maps, count);
    if (p.HW <= 64) return launch_all<64>(p, kind, s, games, maps, count);
    if (p.HW <= 128) return launch_all<128>(p, kind, s, games, maps, count);
    return launch_all<256>(p, kind, s, games, maps, count);
}

// One step launch over n engines of equal planes, obs type and bot fusion, at the
// widest member's workgroup size (a narrower map leaves lanes idle in the game
// logic; every wave still streams outputs).  bots_first: every member's bot games
// take the grid's first segments, then the selfplay games -- workgroups start in
// grid order, so the longest chains (the fused bot after the tick) start first and
// the short selfplay games fill the last round.
static hipError_t step_group(const EngineParams* ps, int n, hipStream_t s, bool bots_first) {
    if (n < 1 || n > MRTS_STEP_GROUP_MAX) return hipErrorInvalidValue;
    const EngineParams& p0 = ps[0];
    const bool fused = p0.fuse_bots != 0;
    int NT = 64;
    for (int i = 0; i < n; i++) {
        const EngineParams& p = ps[i];
        if (p.partial_obs != p0.partial_obs || p.obs_float != p0.obs_float || (p.fuse_bots != 0) != fused) return hipErrorInvalidValue;
        NT = std::max(NT, step_nt(p.HW, fused));
    }
    StepGroup sg{};
    size_t sh = 0;
    for (int i = 0; i < n; i++) {
        EngineParams& e = sg.e[i];
        e = ps[i];
        if (fused) e.early_bot = early_bot_disjoint(e.HW, e.W, NT) ? 1 : 0;   // the layout at this launch's NT
        sh = std::max(sh, fused ? fb_lds_bytes(e.HW, e.W, NT, !e.partial_obs && e.early_bot) : lds_bytes(e.HW, e.W, NT));
    }
    if (sh > 163840) return hipErrorInvalidValue;   // one workgroup's LDS on a CU
    int grid = 0;
    auto seg = [&](int m, int g0, int g1) {
        if (g1 <= g0) return;
        sg.seg_block[sg.nseg] = grid;
        sg.seg_member[sg.nseg] = m;
        sg.seg_game[sg.nseg] = g0;
        sg.nseg++;
        grid += g1 - g0;
    };
    for (int pass = 0; pass < (bots_first ? 2 : 1); pass++)
        for (int i = 0; i < n; i++) {
            const EngineParams& e = sg.e[i];
            if (!bots_first) seg(i, 0, e.G);
            else if (pass == 0) seg(i, e.nsp_games, e.G);
            else seg(i, 0, e.nsp_games);
        }
    sg.seg_block[sg.nseg] = grid;
    if (grid == 0) return hipSuccess;
    if (NT == 64) launch_step<64>(sg, grid, sh, s, p0.partial_obs, p0.obs_float, false);
    else if (NT == 128) launch_step<128>(sg, grid, sh, s, p0.partial_obs, p0.obs_float, fused);
    else launch_step<256>(sg, grid, sh, s, p0.partial_obs, p0.obs_float, fused);
    return hipGetLastError();
}

}  // namespace mrts

extern "C" {
#ifdef MRTS_STAMPS
// experiment builds: copy the stamp rows (every row; rows of workgroups that did not
// run since the last reset are zero) and, with reset != 0, zero them afterwards;
// returns the row count copied
int mrts_debug_stamps(unsigned long long* out, int max_rows, int reset) {
    const int rows = MRTS_STAMP_ROWS < max_rows ? MRTS_STAMP_ROWS : max_rows;
    if (out && rows > 0 &&
        hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(unsigned long long) * MRTS_STAMP_COLS * rows, 0, hipMemcpyDeviceToHost))
        return -1;
    if (reset) {
        static unsigned long long zero[1024][MRTS_STAMP_COLS];
        for (int r = 0; r < MRTS_STAMP_ROWS; r += 1024)
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), zero, sizeof zero, sizeof zero * (r / 1024), hipMemcpyHostToDevice)) return -1;
    }
    return rows;
}
#endif
hipError_t mrts_engine_reset(const EngineParams* p, hipStream_t s, const int32_t* games, const int32_t* maps, int count) {
    return mrts::dispatch(*p, 0, s, games, maps, count);
}
hipError_t mrts_engine_masks(const EngineParams* p, hipStream_t s) { return mrts::dispatch(*p, 1, s, nullptr, nullptr, 0); }
hipError_t mrts_engine_outputs(const EngineParams* p, hipStream_t s) { return mrts::dispatch(*p, 3, s, nullptr, nullptr, 0); }
hipError_t mrts_engine_raw_obs(const EngineParams* p, hipStream_t s, int32_t* raw) {
    const int NT = p->HW <= 64 ? 64 : p->HW <= 128 ? 128 : 256;
    const size_t sh = mrts_engine_lds_bytes(p->HW, p->W);
    if (NT == 64) hipLaunchKernelGGL(mrts::k_raw<64>, dim3(p->G), dim3(64), sh, s, *p, raw);
    else if (NT == 128) hipLaunchKernelGGL(mrts::k_raw<128>, dim3(p->G), dim3(128), sh, s, *p, raw);
    else hipLaunchKernelGGL(mrts::k_raw<256>, dim3(p->G), dim3(256), sh, s, *p, raw);
    return hipGetLastError();
}
hipError_t mrts_engine_step(const EngineParams* p, hipStream_t s) { return mrts::dispatch(*p, 2, s, nullptr, nullptr, 0); }
hipError_t mrts_engine_step_group(const EngineParams* ps, int n, hipStream_t s, int bots_first) {
    return mrts::step_group(ps, n, s, bots_first != 0);
}
size_t mrts_engine_group_lds_bytes(int HW, int W, int fused, int NT, int partial) {
    return fused ? mrts::fb_lds_bytes(HW, W, NT, !partial && mrts::early_bot_disjoint(HW, W, NT)) : mrts::lds_bytes(HW, W, NT);
}
int mrts_engine_step_nt(int HW, int fused) { return mrts::step_nt(HW, fused != 0); }
hipError_t mrts_engine_sample(const int32_t* mask, int n, int hw, int env0, uint64_t seed, uint32_t step, int64_t* act, hipStream_t s) {
    int total = n * hw;
    if (total == 0) return hipSuccess;
    // persistent grid: enough waves to keep every CU streaming, each looping over row groups
    const long long groups = ((long long)total + mrts::SW - 1) / mrts::SW;
    const long long blocks = std::min<long long>((groups + mrts::SWAVES - 1) / mrts::SWAVES, 256 * mrts::SAMPLE_BLOCKS_PER_CU);   // resident blocks
    hipLaunchKernelGGL(mrts::k_sample, dim3((unsigned)blocks), dim3(64 * mrts::SWAVES), 0, s, mask, n, hw, env0, seed, step, act);
    return hipGetLastError();
}
hipError_t mrts_engine_sample_src(const int32_t* mask, const int32_t* src, int n, int hw, int env0, uint64_t seed, uint32_t step,
                                  int64_t* act, hipStream_t s) {
    const long long rows = (long long)n * hw;
    if (rows == 0) return hipSuccess;
    const long long blocks = (rows + 64 * mrts::SR_WAVES - 1) / (64 * mrts::SR_WAVES);
    hipLaunchKernelGGL(mrts::k_sample_src, dim3((unsigned)blocks), dim3(64 * mrts::SR_WAVES), 0, s, mask, src, n, hw, env0, seed, step, act);
    return hipGetLastError();
}
hipError_t mrts_engine_sample_src_group(const mrts_sample_seg* segs, int nseg, uint64_t seed, uint32_t step, hipStream_t s) {
    mrts::SampleGroup g{};
    long long blocks = 0;
    for (int k = 0; k < nseg; k++) {
        const mrts_sample_seg& q = segs[k];
        g.seg[k] = mrts::SampleSeg{q.mask, q.source, q.actions, q.num_envs, q.hw, q.env0};
        blocks += ((long long)q.num_envs * q.hw + 64 * mrts::SR_WAVES - 1) / (64 * mrts::SR_WAVES);
        g.end[k] = blocks;
    }
    g.nseg = nseg;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(mrts::k_sample_src_group, dim3((unsigned)blocks), dim3(64 * mrts::SR_WAVES), 0, s, g, seed, step);
    return hipGetLastError();
}
hipError_t mrts_engine_render(const EngineParams* p, hipStream_t s, int game, int map, int size, uint8_t* rgb) {
    const int nblk = (size * size + 255) / 256;
    hipLaunchKernelGGL(mrts::k_render, dim3(nblk), dim3(256), 0, s, p->cells + (size_t)game * p->cstride, p->map_wall + (size_t)map * p->HW,
                       p->W, p->H, size, rgb);
    return hipGetLastError();
}
int mrts_engine_early_bot_ok(int HW, int W) { return mrts::early_bot_disjoint(HW, W, mrts::step_nt(HW, true)) ? 1 : 0; }
size_t mrts_engine_fused_lds_bytes(int HW, int W, int partial) {
    const int NT = mrts::step_nt(HW, true);
    return mrts::fb_lds_bytes(HW, W, NT, !partial && mrts::early_bot_disjoint(HW, W, NT));
}
size_t mrts_engine_lds_bytes(int HW, int W) {
    int NT = HW <= 64 ? 64 : HW <= 128 ? 128 : 256;
    return mrts::lds_bytes(HW, W, NT);
}
}
