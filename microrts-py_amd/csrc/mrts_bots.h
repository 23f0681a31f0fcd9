// mrts_bots.h -- device code of the scripted opponents, shared by k_bot
// (mrts_bots.hip) and the bot-fused k_step (mrts_engine.hip).
//
// k_bot computes ai2.getAction(1, gs) for every bot game before the step
// kernel issues the tick's actions (JNIGridnetClient.gameStep: ai1.getAction,
// ai2.getAction, issueSafe(pa1), issueSafe(pa2)); k_step then issues the
// PlayerAction it leaves in `botpa` after the agent's.  Restated bots (the Java
// lives in the absent submodule / Coac.jar; rules in oracle/mrts_oracle_ai.c and
// DESIGN.md §4b, which this kernel matches bit for bit):
//   workerRushAI, lightRushAI, POWorkerRush / POLightRush / POHeavyRush /
//   PORangedRush (ai.abstraction.*: AbstractionLayerAI + Move / Harvest / Attack
//   / Train / Build over breadth-first path finding), randomBiasedAI
//   (ai.RandomBiasedAI on a counter-based Philox stream), randomAI
//   (ai.RandomBiasedSingleUnitAI) and coacAI.
//
// Mapping: one WAVEFRONT (64 lanes) per bot game.  The bot's decision logic is
// inherently sequential (units in pgs.units order, the LinkedHashMap of
// abstract actions, a PlayerAction whose ResourceUsage grows as it is built),
// so every lane runs it in lock step on wave-uniform values (LDS stores from
// lane 0; a single wave's LDS operations complete in order).  The parallel
// parts use the lanes: building the uid-ordered unit list, visibility disks,
// pending reservations, and path finding, where lane y holds row y of the
// grid as a bit word and one breadth-first layer is a shift / shuffle / AND.
#ifndef MRTS_BOTS_H
#define MRTS_BOTS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "microrts_amd.h"
#include "mrts_engine.h"
#include "mrts_rules.h"

namespace mrts {
namespace bots {

constexpr int BT = 64;   // one wavefront per bot game


enum { AA_NONE = 0, AA_MOVE, AA_HARVEST, AA_ATTACK, AA_TRAIN, AA_BUILD };

// abstract-action entry = 2 x int4 (LinkedHashMap<Unit, AbstractAction> order):
//   a.x unit uid | a.y kind | completed << 3 | utype << 4 | a.z target uid | a.w destination (packed x, y)
//   b.x harvest base uid | b.y base position (packed x, y; stays valid after the base dies)
__device__ __forceinline__ int pk_xy(int x, int y) { return (x & 0xFFFF) | (y << 16); }
__device__ __forceinline__ int pk_x(int v) { return (int)(short)(v & 0xFFFF); }
__device__ __forceinline__ int pk_y(int v) { return v >> 16; }
__device__ __forceinline__ int aa_kind(int4 a) { return a.y & 7; }
__device__ __forceinline__ int aa_done(int4 a) { return (a.y >> 3) & 1; }
__device__ __forceinline__ int aa_utype(int4 a) { return (a.y >> 4) & 7; }

struct BL {   // LDS of one bot game
    uint32_t* unit;   // the bot's view (PartiallyObservableGameState: hidden units cleared)
    int32_t* uid;
    uint32_t* act;
    int32_t* ucell;   // visible units in pgs.units order (ascending uid)
    int32_t* uuid;
    int32_t* pa;      // PlayerAction under construction: cell | code << 16
    int4* aa;         // [2 * HW] abstract actions
    uint32_t* pend;   // ResourceUsage of the pending assignments: positions + W, bits
    uint32_t* pab;    // the PlayerAction's ResourceUsage positions + W, bits
    uint32_t* vis;    // cells observable by the bot's player (partial obs)
    uint8_t* wall;
    int* sc;          // pending produce cost per player, error bits, [3] = units (workgroup setup)
    uint32_t* fw;     // free-cell words (bot_fw_words)
};

__host__ __device__ inline size_t b16(size_t x) { return (x + 15) & ~(size_t)15; }
// free-cell words: two per 64 cells (one ballot) + a zero word past the last cell
__host__ __device__ inline size_t bot_fw_words(int HW) { return (size_t)(HW + 63) / 64 * 2 + 1; }
// `tail`: where the small arrays (pend, pab, vis, sc, fw) go when the caller keeps
// them apart (the fused k_step's early bot, whose workgroup still reads the
// step's scalars and visibility words while the bot runs); null = behind wall
__host__ __device__ inline size_t bot_tail_bytes(int HW, int W) {
    const size_t posw = (size_t)(HW + 2 * W) / 32 + 1;
    return 2 * b16(4 * posw) + b16(4 * ((size_t)HW / 32 + 1)) + b16(4 * 4) + b16(4 * bot_fw_words(HW));
}
// unit uid act ucell uuid pa + the abstract actions (the fused step's region)
__host__ __device__ inline size_t bot_core_bytes(int HW) { return b16(4 * (size_t)HW) * 6 + b16(32 * (size_t)HW); }
__host__ __device__ inline size_t bot_lds_bytes(int HW, int W) {
    return bot_core_bytes(HW) + b16((size_t)HW) + bot_tail_bytes(HW, W);
}
// own_wall = false: no terrain slot (the fused bot reads the step's terrain in place)
__host__ __device__ inline BL bot_carve(unsigned char* base, int HW, int W, unsigned char* tail = nullptr, bool own_wall = true) {
    BL L;
    size_t o = 0;
    auto take = [&](size_t n) { unsigned char* p = base + o; o += b16(n); return p; };
    const size_t posw = (size_t)(HW + 2 * W) / 32 + 1;
    L.unit = (uint32_t*)take(4 * (size_t)HW);
    L.uid = (int32_t*)take(4 * (size_t)HW);
    L.act = (uint32_t*)take(4 * (size_t)HW);
    L.ucell = (int32_t*)take(4 * (size_t)HW);
    L.uuid = (int32_t*)take(4 * (size_t)HW);
    L.pa = (int32_t*)take(4 * (size_t)HW);
    L.aa = (int4*)take(32 * (size_t)HW);
    L.wall = own_wall ? (uint8_t*)take((size_t)HW) : nullptr;
    if (tail) {
        base = tail;
        o = 0;
    }
    L.pend = (uint32_t*)take(4 * posw);
    L.pab = (uint32_t*)take(4 * posw);
    L.vis = (uint32_t*)take(4 * ((size_t)HW / 32 + 1));
    L.sc = (int*)take(4 * 4);   // pending produce cost per player, error bits, units
    L.fw = (uint32_t*)take(4 * bot_fw_words(HW));
    return L;
}

// wave-uniform scalar state (identical in every lane) + the lane's grid row
struct BS {
    int W, H, HW, player, partial, ai, game;
    uint32_t tick;
    int res[2];
    int n;          // visible units
    int naa;        // abstract actions
    int npa;        // PlayerAction entries
    int pend_res[2];
    int pa_res[2];
    uint32_t frow;  // lane y: free cells of row y (no wall, no visible unit)
    uint32_t rurow; // lane y: PlayerAction positions in row y (path finding's ResourceUsage)
    // n <= 64: the unit list lives in registers, entry k in lane k (0 / INT_MIN past the list)
    int kcell;      // cell of unit k
    int kuid;       // its uid
    uint32_t kunit; // its unit word (the bot's view)
    uint32_t kact;  // its pending action word
    int kenemy;     // list index of unit k's closest enemy (-1: none), for the behaviours
    // naa <= 64: abstract action k (both int4 words) in lane k; the LDS list is kept too
    int4 kA, kB;
#ifdef MRTS_STAMPS
    // the bot's counters (experiment builds), stamped once at its end (columns 16-19)
    unsigned long long c_entries, c_searches, c_ticks, c_rounds;   // written once, at the bot's end
#endif
};

// one unit of the list, read from the registers (or LDS past 64 units)
struct URef {
    int k;          // list index (pgs.units order)
    int c, uid;
    uint32_t u;     // unit word
};

// lane of the bot's wavefront: k_bot is one wave; in the fused k_step any wave
// of the workgroup may run the bot (the launch rotates it over the SIMDs)
__device__ __forceinline__ int blane() { return (int)(threadIdx.x & 63u); }
__device__ __forceinline__ bool lane0() { return blane() == 0; }
__device__ __forceinline__ int iabs(int a) { return a < 0 ? -a : a; }

__device__ __forceinline__ bool in_map(const BS& S, int x, int y) { return x >= 0 && y >= 0 && x < S.W && y < S.H; }
__device__ __forceinline__ bool v_free(const BS& S, const BL& L, int x, int y) {   // GameState.free
    if (!in_map(S, x, y)) return false;
    int c = y * S.W + x;
    return !L.wall[c] && L.unit[c] == 0;
}

// ---- cross-lane moves without LDS: DPP and scalar lane reads ---------------------
// The bot is one wave whose decisions are a long chain of dependent steps, so
// every cross-lane step is on the critical path: ds_bpermute (__shfl) costs an
// LDS round trip, DPP and v_readlane a few VALU cycles.
__device__ __forceinline__ uint32_t from_lane_below(uint32_t v) {   // lane l <- lane l-1, lane 0 <- 0 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_lane_above(uint32_t v) {   // lane l <- lane l+1, lane 63 <- 0 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ int lane_value(int v, int lane) {   // v of lane `lane` (wave-uniform index)
    return __builtin_amdgcn_readlane(v, lane);
}
// wave-wide unsigned minimum: DPP prefix minima inside each 16-lane row, then the four rows' last lanes
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    const uint32_t a = (uint32_t)lane_value((int)v, 15), b = (uint32_t)lane_value((int)v, 31);
    const uint32_t c = (uint32_t)lane_value((int)v, 47), d = (uint32_t)lane_value((int)v, 63);
    return min(min(a, b), min(c, d));
}

// uid -> cell in the bot's view, -1 if absent: one compare per lane over the
// uid-ordered list (registers when it fits the wave), a ballot and a lane read.
// With `act`: the unit's pending action word too.
__device__ __forceinline__ int cell_of_uid(const BS& S, const BL& L, int uid, uint32_t* act = nullptr) {
    if (S.n <= BT) {
        const unsigned long long m = __ballot(S.kuid == uid);
        if (!m) return -1;
        if (act) *act = (uint32_t)lane_value((int)S.kact, __builtin_ctzll(m));
        return lane_value(S.kcell, __builtin_ctzll(m));
    }
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + blane();
        const unsigned long long m = __ballot(k < S.n && L.uuid[k] == uid);
        if (m) {
            const int c = L.ucell[base + __builtin_ctzll(m)];
            if (act) *act = L.act[c];
            return c;
        }
    }
    return -1;
}

// ---- wave-parallel scans of the unit list (results identical in every lane) ----
// Predicates see (cell, unit word, action word) of one list entry per lane.
__device__ __forceinline__ void list_entry(const BS& S, const BL& L, int k, int& c, uint32_t& u, uint32_t& a) {
    if (S.n <= BT) {
        c = S.kcell;
        u = S.kunit;
        a = S.kact;
    } else {
        c = k < S.n ? L.ucell[k] : 0;
        u = k < S.n ? L.unit[c] : 0u;
        a = k < S.n ? L.act[c] : 0u;
    }
}
// The first unit in pgs.units order (a serial `d < best` scan) among those
// `want` selects minimising the Manhattan distance to (x, y): min over the
// packed key (distance << 16 | list index) across the lanes.  -1 if none;
// *dist = that distance.
template <typename F>
__device__ __forceinline__ int closest_index(const BS& S, const BL& L, int x, int y, F want, int* dist = nullptr);
__device__ __forceinline__ URef ref_at(const BS& S, const BL& L, int k) {
    URef r;
    r.k = k;
    if (S.n <= BT) {
        r.c = lane_value(S.kcell, k);
        r.uid = lane_value(S.kuid, k);
        r.u = (uint32_t)lane_value((int)S.kunit, k);
    } else {
        r.c = L.ucell[k];
        r.uid = L.uuid[k];
        r.u = L.unit[r.c];
    }
    return r;
}
template <typename F>
__device__ __forceinline__ int closest_unit(const BS& S, const BL& L, int x, int y, F want, int* dist = nullptr) {
    const int k = closest_index(S, L, x, y, want, dist);
    return k < 0 ? -1 : (S.n <= BT ? lane_value(S.kcell, k) : L.ucell[k]);
}
// list index of the closest unit `want` selects (see closest_unit), -1 if none
template <typename F>
__device__ __forceinline__ int closest_index(const BS& S, const BL& L, int x, int y, F want, int* dist) {
    uint32_t key = 0xFFFFFFFFu;
    for (int k = blane(); k < S.n; k += BT) {
        int c;
        uint32_t u, a;
        list_entry(S, L, k, c, u, a);
        if (!want(c, u, a)) continue;
        const uint32_t d = (uint32_t)(iabs(c % S.W - x) + iabs(c / S.W - y));
        const uint32_t kk = (d << 16) | (uint32_t)k;
        key = kk < key ? kk : key;
    }
    key = wave_min_u32(key);
    if (key == 0xFFFFFFFFu) return -1;
    if (dist) *dist = (int)(key >> 16);
    return (int)(key & 0xFFFFu);
}
// body(cell) for every unit of the list `want` selects, in pgs.units order.
// `want` must not depend on what `body` changes (abstract actions, the PlayerAction).
template <typename P, typename F>
__device__ __forceinline__ void for_each_unit(const BS& S, const BL& L, P want, F body) {
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + blane();
        int c;
        uint32_t u, a;
        list_entry(S, L, k, c, u, a);
        unsigned long long m = __ballot(k < S.n && want(c, u, a));
        while (m) {
            const int j = __builtin_ctzll(m);
            m &= m - 1ull;
            body(ref_at(S, L, base + j));
        }
    }
}
// number of units `want` selects
template <typename F>
__device__ __forceinline__ int count_where(const BS& S, const BL& L, F want) {
    int n = 0;
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + blane();
        int c;
        uint32_t u, a;
        list_entry(S, L, k, c, u, a);
        n += __popcll(__ballot(k < S.n && want(c, u, a)));
    }
    return n;
}
// list index of the idx-th unit (pgs.units order) `want` selects, -1 if fewer
template <typename F>
__device__ __forceinline__ int nth_index(const BS& S, const BL& L, int idx, F want) {
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + blane();
        int c;
        uint32_t u, a;
        list_entry(S, L, k, c, u, a);
        unsigned long long m = __ballot(k < S.n && want(c, u, a));
        const int cnt = __popcll(m);
        if (idx < cnt) {
            for (int t = 0; t < idx; t++) m &= m - 1ull;
            return base + __builtin_ctzll(m);
        }
        idx -= cnt;
    }
    return -1;
}

// ---- ResourceUsage ----------------------------------------------------------
struct RU {
    int pos;    // unchecked x + y*W + offset, or INT_MIN for none
    int res[2];
};
__device__ __forceinline__ RU usage(const BS& S, int c, int code, int owner) {   // UnitAction.resourceUsage
    RU r{-0x7fffffff, {0, 0}};
    const int t = code_type(code);
    if (t == A_MOVE || t == A_PRODUCE) {
        const int d = code_param(code);   // selects, not an indexed local array (scratch)
        r.pos = c + (d == 0 ? -S.W : d == 1 ? 1 : d == 2 ? S.W : -1);
        if (t == A_PRODUCE) {
            if (owner == 0) r.res[0] = ut_cost(code_utype(code));
            else if (owner == 1) r.res[1] = ut_cost(code_utype(code));
        }
    }
    return r;
}
__device__ __forceinline__ bool bit_at(const uint32_t* b, int i) { return (b[i >> 5] >> (i & 31)) & 1u; }
// ResourceUsage.consistentWith(another = bits + res, gs)
__device__ __forceinline__ bool consistent(const BS& S, const RU& r, const uint32_t* bits, const int* res) {
    if (r.pos != -0x7fffffff && bit_at(bits, r.pos + S.W)) return false;
    for (int i = 0; i < 2; i++) {
        int s = r.res[i] + res[i];
        if (s > 0 && s > S.res[i]) return false;
    }
    return true;
}

// GameState.isUnitActionAllowed on the bot's state
__device__ __forceinline__ bool allowed(const BS& S, const BL& L, int c, int code) {
    if (code_type(code) == A_MOVE) {
        int n = nb_cell(Grid{S.W, S.H, S.HW}, c, code_param(code));
        if (n < 0 || L.wall[n] || L.unit[n] != 0) return false;
    }
    RU r = usage(S, c, code, u_owner(L.unit[c]));
    return consistent(S, r, L.pend, S.pend_res);
}

// PlayerAction.addUnitAction + ResourceUsage.merge
__device__ __forceinline__ void pa_add(BS& S, const BL& L, int c, int code) {
    RU r = usage(S, c, code, u_owner(L.unit[c]));
    if (lane0()) {
        L.pa[S.npa] = c | (code << 16);
        if (r.pos != -0x7fffffff) {
            int i = r.pos + S.W;
            L.pab[i >> 5] |= 1u << (i & 31);
        }
    }
    S.npa++;
    S.pa_res[0] += r.res[0];
    S.pa_res[1] += r.res[1];
    if (r.pos != -0x7fffffff && r.pos >= 0 && r.pos < S.HW && blane() == r.pos / S.W)
        S.rurow |= 1u << (r.pos % S.W);
}

// ---- AStarPathFinding.findPathToPositionInRange (restated: DESIGN.md §4b) ----
// Breadth-first layers grow from the goal set (free cells within `range` of
// the target) over free cells; the first layer that touches a free neighbour
// of the start decides the move, ties UP, RIGHT, DOWN, LEFT.  -1 = null.
__device__ __forceinline__ int pf_dir_search(const BS& S, int sc, int tx, int ty, int range) {
    const int lane = blane(), sx = sc % S.W, sy = sc / S.W, r2 = range * range;
    if ((sx - tx) * (sx - tx) + (sy - ty) * (sy - ty) <= r2) return -1;
    const uint32_t rowmask = S.W == 32 ? 0xFFFFFFFFu : ((1u << S.W) - 1u);
    uint32_t fr = 0, goal = 0;
    if (lane < S.H) {
        fr = S.frow & ~S.rurow;
        const int dy = lane - ty, rem = r2 - dy * dy;
        if (rem >= 0) {
            int s = 0;
            while ((s + 1) * (s + 1) <= rem) s++;
            const int x0 = max(0, tx - s), x1 = min(S.W - 1, tx + s);
            if (x0 <= x1) goal = (x1 - x0 == 31 ? 0xFFFFFFFFu : ((1u << (x1 - x0 + 1)) - 1u)) << x0;
        }
        goal &= fr;
    }
    // the start's four neighbours as bits of their rows: one ballot per layer
    // tells whether the front reached any of them (the direction is then read once)
    uint32_t nbr = 0;
    if (lane == sy) nbr = ((sx + 1 < S.W) ? 1u << (sx + 1) : 0u) | (sx > 0 ? 1u << (sx - 1) : 0u);
    if (lane == sy - 1 || lane == sy + 1) nbr = 1u << sx;
    const uint32_t frm = fr & rowmask;
    auto grow_of = [&](uint32_t f, uint32_t sn) {   // the next layer: rows y-1 and y+1 of f (rows >= H hold no free cell)
        return ((f << 1) | (f >> 1) | from_lane_below(f) | from_lane_above(f)) & frm & ~sn;
    };
    auto first_dir = [&](uint32_t f) {   // the layer touches a neighbour: ties UP, RIGHT, DOWN, LEFT
        const uint32_t rU = (uint32_t)lane_value((int)f, max(sy - 1, 0)), rC = (uint32_t)lane_value((int)f, sy),
                       rD = (uint32_t)lane_value((int)f, min(sy + 1, 63));
        if (sy > 0 && ((rU >> sx) & 1u)) return 0;
        if (sx + 1 < S.W && ((rC >> (sx + 1)) & 1u)) return 1;
        if (sy + 1 < S.H && ((rD >> sx) & 1u)) return 2;
        return 3;
    };
    // four layers per round, one branch for "a layer touched a neighbour" and one for
    // "the front died": the same first touching layer and the same null path as one
    // layer at a time (a layer after an empty one is empty too)
    uint32_t seen = goal, front = goal;
    for (int it = 0; it <= S.HW; it += 4) {
#ifdef MRTS_STAMPS
        const_cast<BS&>(S).c_rounds++;   // four-layer rounds
#endif
        const uint32_t g1 = grow_of(front, seen), s1 = seen | g1;
        const uint32_t g2 = grow_of(g1, s1), s2 = s1 | g2;
        const uint32_t g3 = grow_of(g2, s2), s3 = s2 | g3;
        const uint32_t g4 = grow_of(g3, s3);
        const unsigned long long t0 = __ballot((front & nbr) != 0), t1 = __ballot((g1 & nbr) != 0);
        const unsigned long long t2 = __ballot((g2 & nbr) != 0), t3 = __ballot((g3 & nbr) != 0);
        if (t0 | t1 | t2 | t3) return first_dir(t0 ? front : t1 ? g1 : t2 ? g2 : g3);
        if (!__ballot(g4 != 0)) return -1;
        seen = s3 | g4;
        front = g4;
    }
    return -1;
}

// (experiment builds: the searches' count and summed time per bot)
__device__ __forceinline__ int pf_dir(const BS& S, int sc, int tx, int ty, int range) {
#ifdef MRTS_STAMPS
    const unsigned long long t0 = wall_clock64();
    const int d = pf_dir_search(S, sc, tx, ty, range);
    const_cast<BS&>(S).c_searches++;
    const_cast<BS&>(S).c_ticks += wall_clock64() - t0;
    return d;
#else
    return pf_dir_search(S, sc, tx, ty, range);
#endif
}

// ---- abstract actions ----------------------------------------------------------
// LinkedHashMap<Unit, AbstractAction> in insertion order: the LDS list is the
// record; while it holds <= 64 entries, entry k also lives in lane k's kA / kB,
// and lookups are one ballot / lane read.
__device__ __forceinline__ int find_aa(const BS& S, const BL& L, int uid) {   // first entry of the unit, lane-parallel
    if (S.naa <= BT) {
        const unsigned long long m = __ballot(blane() < S.naa && S.kA.x == uid);
        return m ? __builtin_ctzll(m) : -1;
    }
    for (int base = 0; base < S.naa; base += BT) {
        const int k = base + blane();
        const unsigned long long m = __ballot(k < S.naa && L.aa[2 * k].x == uid);
        if (m) return base + __builtin_ctzll(m);
    }
    return -1;
}
__device__ __forceinline__ int4 lane_int4(int4 v, int k) {
    return make_int4(lane_value(v.x, k), lane_value(v.y, k), lane_value(v.z, k), lane_value(v.w, k));
}
__device__ __forceinline__ void aa_entry(const BS& S, const BL& L, int k, int4& a, int4& b) {
    if (S.naa <= BT) {
        a = lane_int4(S.kA, k);
        b = lane_int4(S.kB, k);
    } else {
        a = L.aa[2 * k];
        b = L.aa[2 * k + 1];
    }
}
__device__ __forceinline__ void aa_put(BS& S, const BL& L, int4 a, int4 b) {   // actions.put(u, aa)
    int k = find_aa(S, L, a.x);
    if (k < 0) {
        if (S.naa >= S.HW) {   // more live entries than cells: cannot happen on legal states
            if (lane0()) L.sc[2] |= MRTS_ERR_BOT_OVERFLOW;
            return;
        }
        k = S.naa++;
    }
    if (blane() == k) {
        S.kA = a;
        S.kB = b;
    }
    if (lane0()) {
        L.aa[2 * k] = a;
        L.aa[2 * k + 1] = b;
    }
}
__device__ __forceinline__ void ab_move(BS& S, const BL& L, int uid, int x, int y) {
    aa_put(S, L, make_int4(uid, AA_MOVE, -1, pk_xy(x, y)), make_int4(-1, 0, 0, 0));
}
__device__ __forceinline__ void ab_train(BS& S, const BL& L, int uid, int t) {
    aa_put(S, L, make_int4(uid, AA_TRAIN | (t << 4), -1, 0), make_int4(-1, 0, 0, 0));
}
__device__ __forceinline__ void ab_build(BS& S, const BL& L, int uid, int t, int x, int y) {
    aa_put(S, L, make_int4(uid, AA_BUILD | (t << 4), -1, pk_xy(x, y)), make_int4(-1, 0, 0, 0));
}
__device__ __forceinline__ void ab_harvest(BS& S, const BL& L, int uid, int res_uid, int base_uid, int base_cell) {
    aa_put(S, L, make_int4(uid, AA_HARVEST, res_uid, 0), make_int4(base_uid, pk_xy(base_cell % S.W, base_cell / S.W), 0, 0));
}
__device__ __forceinline__ void ab_attack(BS& S, const BL& L, int uid, int target_uid) {
    aa_put(S, L, make_int4(uid, AA_ATTACK, target_uid, 0), make_int4(-1, 0, 0, 0));
}

__device__ __forceinline__ int adj_dir(int ux, int uy, int x, int y) {
    if (x == ux && y == uy - 1) return 0;
    if (x == ux + 1 && y == uy) return 1;
    if (x == ux && y == uy + 1) return 2;
    if (x == ux - 1 && y == uy) return 3;
    return -1;
}

__device__ __forceinline__ int train_score(const BS& S, const BL& L, int x, int y, int type, int player) {   // Train.score
    int dist = 0;   // stays 0 when nothing qualifies
    closest_unit(S, L, x, y, [&](int, uint32_t o, uint32_t) {
        return ut_can_harvest(type) ? u_type(o) == RESOURCE : (u_owner(o) >= 0 && u_owner(o) != player);
    }, &dist);
    return -dist;
}

__device__ __forceinline__ bool aa_completed(const BS& S, const BL& L, int4 a, int cu) {
    switch (aa_kind(a)) {
    case AA_MOVE: return cu % S.W == pk_x(a.w) && cu / S.W == pk_y(a.w);
    case AA_HARVEST:
    case AA_ATTACK: return cell_of_uid(S, L, a.z) < 0;
    default: return aa_done(a) != 0;
    }
}

// AbstractAction.execute: action code, or -1 for null; may set `completed`
__device__ __forceinline__ int aa_execute(const BS& S, const BL& L, int4& a, int4 b, int cu) {
    const uint32_t u = L.unit[cu];
    const int ux = cu % S.W, uy = cu / S.W;
    switch (aa_kind(a)) {
    case AA_MOVE: {
        int d = pf_dir(S, cu, pk_x(a.w), pk_y(a.w), 0);
        if (d < 0) return -1;
        int code = code_make(A_MOVE, d, 0);
        return allowed(S, L, cu, code) ? code : -1;
    }
    case AA_HARVEST: {
        int tx, ty;
        if (u_res(u) == 0) {
            int tc = cell_of_uid(S, L, a.z);
            tx = tc % S.W;
            ty = tc / S.W;
        } else {
            tx = pk_x(b.y);
            ty = pk_y(b.y);
        }
        int d = pf_dir(S, cu, tx, ty, 1);
        if (d >= 0) {
            int code = code_make(A_MOVE, d, 0);
            return allowed(S, L, cu, code) ? code : -1;
        }
        int ad = adj_dir(ux, uy, tx, ty);
        if (ad < 0) return -1;
        return code_make(u_res(u) == 0 ? A_HARVEST : A_RETURN, ad, 0);
    }
    case AA_ATTACK: {
        int tc = cell_of_uid(S, L, a.z);
        int dx = tc % S.W - ux, dy = tc / S.W - uy, r = ut_range(u_type(u));
        if (dx * dx + dy * dy <= r * r)
            return code_make(A_ATTACK, (dy + MRTS_ATTACK_GRID / 2) * MRTS_ATTACK_GRID + (dx + MRTS_ATTACK_GRID / 2), 0);
        int d = pf_dir(S, cu, tc % S.W, tc / S.W, r);
        if (d < 0) return -1;
        int code = code_make(A_MOVE, d, 0);
        return allowed(S, L, cu, code) ? code : -1;
    }
    case AA_TRAIN: {
        const int t = aa_utype(a);
        int best = -1, bs = -1;
        for (int d = 0; d < 4; d++) {
            int x = ux + dir_dx(d), y = uy + dir_dy(d);
            if (!v_free(S, L, x, y)) continue;
            int sc = train_score(S, L, x, y, t, u_owner(u));
            if (sc > bs || best == -1) {
                bs = sc;
                best = d;
            }
        }
        a.y |= 1 << 3;   // completed = true
        if (best < 0) return -1;
        int code = code_make(A_PRODUCE, best, t);
        return allowed(S, L, cu, code) ? code : -1;
    }
    case AA_BUILD: {
        const int bx = pk_x(a.w), by = pk_y(a.w);
        int d = pf_dir(S, cu, bx, by, 1);
        if (d >= 0) {
            int code = code_make(A_MOVE, d, 0);
            return allowed(S, L, cu, code) ? code : -1;
        }
        int ad = adj_dir(ux, uy, bx, by);
        if (ad < 0) return -1;
        int code = code_make(A_PRODUCE, ad, aa_utype(a));
        if (!allowed(S, L, cu, code)) return -1;
        a.y |= 1 << 3;
        return code;
    }
    }
    return -1;
}

// AbstractionLayerAI.translateActions (fillWithNones(gs, p, 1) is k_step's phase 3)
// With the unit list and the abstract actions in registers (<= 64 each): whether
// an entry is dropped (its unit or target gone, or completed) and whether its unit
// is idle depend on the fixed state only, so every entry decides that in its own
// lane (its unit's and its target's cells found in one pass over the list); only
// the idle units' AbstractAction.execute, whose PlayerAction ResourceUsage grows
// entry by entry, walks the entries in order; the kept entries are then written
// back lane-parallel in their order.
__device__ __forceinline__ void translate_actions_lanes(BS& S, const BL& L) {
    const int lane = blane();
    const bool valid = lane < S.naa;
    int4 a = S.kA;
    const int4 b = S.kB;
    int cu = -1, tc = -1;
    uint32_t act = 0;
    for (int j = 0; j < S.n; j++) {   // uid -> cell of the entry's unit and of its target
        const int uj = lane_value(S.kuid, j), cj = lane_value(S.kcell, j);
        const uint32_t aj = (uint32_t)lane_value((int)S.kact, j);
        if (uj == a.x) {
            cu = cj;
            act = aj;
        }
        if (uj == a.z) tc = cj;
    }
    bool done = false;   // aa_completed
    switch (aa_kind(a)) {
    case AA_MOVE: done = cu % S.W == pk_x(a.w) && cu / S.W == pk_y(a.w); break;
    case AA_HARVEST:
    case AA_ATTACK: done = tc < 0; break;
    default: done = aa_done(a) != 0;
    }
    const bool keep = valid && cu >= 0 && !done;
    unsigned long long ex = __ballot(keep && act == 0);
    while (ex) {   // the idle units' execute, in LinkedHashMap order
        const int k = __builtin_ctzll(ex);
        ex &= ex - 1ull;
        int4 ak = lane_int4(a, k);
        const int4 bk = lane_int4(b, k);
        const int cuk = lane_value(cu, k);
#ifdef MRTS_STAMPS
        S.c_entries++;   // executed entries
#endif
        const int code = aa_execute(S, L, ak, bk, cuk);
        if (code >= 0) {
            RU r = usage(S, cuk, code, S.player);
            if (consistent(S, r, L.pab, S.pa_res)) pa_add(S, L, cuk, code);
        }
        if (lane == k) a = ak;   // execute may mark it completed
    }
    const unsigned long long km = __ballot(keep);
    if (keep) {
        const int pos = __popcll(km & ((1ull << lane) - 1ull));
        L.aa[2 * pos] = a;
        L.aa[2 * pos + 1] = b;
    }
    S.naa = __popcll(km);   // (the register copy is stale from here on: only the LDS list is written back)
}

__device__ __forceinline__ void translate_actions(BS& S, const BL& L) {
    if (S.n <= BT && S.naa <= BT) {
        translate_actions_lanes(S, L);
        return;
    }
    int w = 0;
    const int n0 = S.naa;
    for (int k = 0; k < n0; k++) {
        int4 a, b;
        aa_entry(S, L, k, a, b);
        uint32_t act = 0;
        const int cu = cell_of_uid(S, L, a.x, &act);
        const bool del = cu < 0 || aa_completed(S, L, a, cu);
        if (!del && act == 0) {
            const int code = aa_execute(S, L, a, b, cu);
            if (code >= 0) {
                RU r = usage(S, cu, code, S.player);
                if (consistent(S, r, L.pab, S.pa_res)) pa_add(S, L, cu, code);
            }
        }
        if (!del) {
            if (lane0()) {
                L.aa[2 * w] = a;
                L.aa[2 * w + 1] = b;
            }
            w++;
        }
    }
    S.naa = w;   // (the register copy is stale from here on: only the LDS list is written back)
}

// ---- behaviours ------------------------------------------------------------------
// closest enemy of a unit: the table the bot builds before the behaviours (rush
// family, coacAI), or a wave-parallel scan
__device__ __forceinline__ int closest_enemy_index(const BS& S, const BL& L, const URef& w, bool table = true) {
    if (table) return S.n <= BT ? lane_value(S.kenemy, w.k) : L.pa[w.k];
    const int me = u_owner(w.u);
    return closest_index(S, L, w.c % S.W, w.c / S.W, [&](int, uint32_t u, uint32_t) {
        const int o = u_owner(u);
        return o >= 0 && o != me;
    });
}
__device__ __forceinline__ int closest_of_index(const BS& S, const BL& L, const URef& w, bool want_resource) {
    const int me = u_owner(w.u);
    return closest_index(S, L, w.c % S.W, w.c / S.W, [&](int, uint32_t o, uint32_t) {
        return want_resource ? u_type(o) == RESOURCE : (ut_is_stockpile(u_type(o)) && u_owner(o) == me);
    }, nullptr);
}

// meleeUnitBehavior (+ PO* exploration: nearest cell the player cannot observe)
__device__ __forceinline__ void melee_behavior(BS& S, const BL& L, const URef& w, bool po) {
    const int e = closest_enemy_index(S, L, w);
    if (e >= 0) {
        ab_attack(S, L, w.uid, ref_at(S, L, e).uid);
        return;
    }
    if (!(po && S.partial)) return;
    const int ux = w.c % S.W, uy = w.c / S.W;
    // first minimum in row-major scan order = min over (d^2 << 16 | cell); d^2 <= 32^2 + 64^2
    uint32_t key = 0xFFFFFFFFu;
    for (int c = blane(); c < S.HW; c += BT) {
        if (bit_at(L.vis, c)) continue;
        const int x = c % S.W, y = c / S.W;
        const uint32_t kk = ((uint32_t)((ux - x) * (ux - x) + (uy - y) * (uy - y)) << 16) | (uint32_t)c;
        key = kk < key ? kk : key;
    }
    key = wave_min_u32(key);
    if (key != 0xFFFFFFFFu) {
        const int c = (int)(key & 0xFFFFu);
        ab_move(S, L, w.uid, c % S.W, c / S.W);
    }
}

// harvest(closest resource, closest own base) unless already harvesting those
__device__ __forceinline__ void harvest_behavior(BS& S, const BL& L, const URef& w) {
    const int ri = closest_of_index(S, L, w, true), bi = closest_of_index(S, L, w, false);
    if (ri < 0 || bi < 0) return;
    const URef r = ref_at(S, L, ri), b = ref_at(S, L, bi);
    const int k = find_aa(S, L, w.uid);
    if (k >= 0) {
        int4 a, bb;
        aa_entry(S, L, k, a, bb);
        if (aa_kind(a) == AA_HARVEST && a.z == r.uid && bb.x == b.uid) return;
    }
    ab_harvest(S, L, w.uid, r.uid, b.uid, b.c);
}

// AbstractionLayerAI.findBuildingPosition
// building positions reserved by this getAction (a base and a barracks at most), in registers
struct Rsv {
    int a, b, n;
};
__device__ __forceinline__ int find_building_position(const BS& S, const BL& L, const Rsv& rs, int dx, int dy) {
    const int Lmax = max(S.W, S.H);
    for (int l = 1; l < Lmax; l++) {
        for (int side = 0; side < 4; side++) {
            for (int k = -l; k <= l; k++) {
                int x, y;
                if (side == 0) { y = dy - l; x = dx + k; if (y < 0) break; }
                else if (side == 1) { x = dx + l; y = dy + k; if (x >= S.W) break; }
                else if (side == 2) { y = dy + l; x = dx + k; if (y >= S.H) break; }
                else { x = dx - l; y = dy + k; if (x < 0) break; }
                if (!in_map(S, x, y)) continue;
                const int pos = x + y * S.W;
                const bool taken = (rs.n > 0 && rs.a == pos) || (rs.n > 1 && rs.b == pos);
                if (!taken && v_free(S, L, x, y)) return pos;
            }
        }
    }
    return -1;
}

__device__ __forceinline__ void build_if_not_already(BS& S, const BL& L, const URef& w, int type, Rsv& rs) {
    const int k = find_aa(S, L, w.uid);
    if (k >= 0) {
        int4 a, b;
        aa_entry(S, L, k, a, b);
        if (aa_kind(a) == AA_BUILD && aa_utype(a) == type) return;
    }
    const int pos = find_building_position(S, L, rs, w.c % S.W, w.c / S.W);
    ab_build(S, L, w.uid, type, pos % S.W, pos / S.W);   // C/Java division: -1 -> (-1, 0)
    if (rs.n == 0) rs.a = pos;
    else rs.b = pos;
    rs.n++;
}

// unit selectors for for_each_unit: the player's idle units of a type / idle army units
__device__ __forceinline__ auto idle_own(const BS& S, const BL& L, int type) {
    return [&S, type](int, uint32_t u, uint32_t a) { return u_type(u) == type && u_owner(u) == S.player && a == 0; };
}
__device__ __forceinline__ auto idle_own_army(const BS& S, const BL& L) {
    return [&S](int, uint32_t u, uint32_t a) {
        const int t = u_type(u);
        return ut_can_attack(t) && !ut_can_harvest(t) && u_owner(u) == S.player && a == 0;
    };
}

__device__ __forceinline__ int count_units(const BS& S, const BL& L, int type, bool own) {
    return count_where(S, L, [&](int, uint32_t o, uint32_t) {
        return u_type(o) == type && (own ? u_owner(o) == S.player : (u_owner(o) >= 0 && u_owner(o) != S.player));
    });
}

// WorkerRush / LightRush / HeavyRush / RangedRush (+ PO*)
__device__ __forceinline__ void behaviours_parallel(BS& S, const BL& L, int army, bool po, bool coac);
// The rush family's behaviours unit by unit (more units or abstract actions than a
// wave has lanes; behaviours_parallel otherwise).  bot_game translates afterwards.
__device__ __forceinline__ void rush_serial(BS& S, const BL& L, int army, bool po) {
    const int p = S.player, res = p ? S.res[1] : S.res[0];
    const int nworkers = count_units(S, L, WORKER, true), nbases = count_units(S, L, BASE, true),
              nbarracks = count_units(S, L, BARRACKS, true);
    const bool tr = army == WORKER ? res >= ut_cost(WORKER) : nworkers < 1 && res >= ut_cost(WORKER);
    if (tr) for_each_unit(S, L, idle_own(S, L, BASE), [&](const URef& b) { ab_train(S, L, b.uid, WORKER); });   // bases
    if (army != WORKER && res >= ut_cost(army))                                                                // barracks
        for_each_unit(S, L, idle_own(S, L, BARRACKS), [&](const URef& b) { ab_train(S, L, b.uid, army); });
    for_each_unit(S, L, idle_own_army(S, L), [&](const URef& m) { melee_behavior(S, L, m, po); });            // melee units
    // workers, busy ones included (the list is the tail of the unit list walk)
    auto own_worker = [&](int, uint32_t u, uint32_t) { return ut_can_harvest(u_type(u)) && u_owner(u) == p; };
    const int nf = count_where(S, L, own_worker);
    if (nf > 0) {
        Rsv reserved{0, 0, 0};
        int used = 0, head = 0;   // head: workers taken off the free list
        auto worker = [&](int idx) { return ref_at(S, L, nth_index(S, L, idx, own_worker)); };   // idx-th own worker
        if (nbases == 0 && head < nf && res >= ut_cost(BASE) + used) {
            build_if_not_already(S, L, worker(head++), BASE, reserved);
            used += ut_cost(BASE);
        }
        if (army == WORKER) {
            if (head < nf) harvest_behavior(S, L, worker(head++));
            for (int k = head; k < nf; k++) melee_behavior(S, L, worker(k), po);
        } else {
            if (nbarracks == 0 && res >= ut_cost(BARRACKS) + used && head < nf) {
                build_if_not_already(S, L, worker(head++), BARRACKS, reserved);
                used += ut_cost(BARRACKS);
            }
            for (int k = head; k < nf; k++) harvest_behavior(S, L, worker(k));
        }
    }
}


// coacAI: CoacAI's published strategy, restated (oracle/mrts_oracle_ai.c
// coac_get_action; its free choices are fixed by league.db's outcomes)
constexpr int COAC_HARVESTERS_PER_BASE = 2, COAC_EXTRA_WORKERS = 2, COAC_BARRACKS_MIN_WORKERS = 2, COAC_DEFENSE_RADIUS = 8;
// (unit by unit, as rush_serial)
__device__ __forceinline__ void coac_serial(BS& S, const BL& L) {
    const int p = S.player, res = p ? S.res[1] : S.res[0];
    const int nworkers = count_units(S, L, WORKER, true), nbases = count_units(S, L, BASE, true),
              nbarracks = count_units(S, L, BARRACKS, true);
    if (nworkers < COAC_HARVESTERS_PER_BASE * nbases + COAC_EXTRA_WORKERS && res >= ut_cost(WORKER))     // bases
        for_each_unit(S, L, idle_own(S, L, BASE), [&](const URef& b) { ab_train(S, L, b.uid, WORKER); });
    const int t = count_units(S, L, LIGHT, false) > count_units(S, L, RANGED, false) + count_units(S, L, HEAVY, false) ? HEAVY : RANGED;
    if (res >= ut_cost(t))                                                                                    // barracks
        for_each_unit(S, L, idle_own(S, L, BARRACKS), [&](const URef& b) { ab_train(S, L, b.uid, t); });
    for_each_unit(S, L, idle_own_army(S, L), [&](const URef& m) { melee_behavior(S, L, m, false); });       // army
    auto own_worker = [&](int, uint32_t u, uint32_t) { return ut_can_harvest(u_type(u)) && u_owner(u) == p; };
    const int nf = count_where(S, L, own_worker);
    if (nf > 0) {
        Rsv reserved{0, 0, 0};
        int used = 0, head = 0;
        auto worker = [&](int idx) { return ref_at(S, L, nth_index(S, L, idx, own_worker)); };
        if (nbases == 0 && head < nf && res >= ut_cost(BASE) + used) {
            build_if_not_already(S, L, worker(head++), BASE, reserved);
            used += ut_cost(BASE);
        }
        if (nbarracks == 0 && res >= ut_cost(BARRACKS) + used && head < nf && nworkers >= COAC_BARRACKS_MIN_WORKERS) {
            build_if_not_already(S, L, worker(head++), BARRACKS, reserved);
            used += ut_cost(BARRACKS);
        }
        const int nh = COAC_HARVESTERS_PER_BASE * (nbases > 0 ? nbases : 1);
        for (int k = head; k < nf; k++) {
            const URef w = worker(k);
            if (k - head < nh) {
                harvest_behavior(S, L, w);
                continue;
            }
            // defenders: the closest enemy when it is near the worker's closest own base
            const int ei = closest_enemy_index(S, L, w);
            if (ei < 0) continue;
            const int bi = closest_of_index(S, L, w, false);
            const URef e = ref_at(S, L, ei);
            const int bc = bi < 0 ? -1 : ref_at(S, L, bi).c;
            if (bi < 0 || iabs(bc % S.W - e.c % S.W) + iabs(bc / S.W - e.c / S.W) <= COAC_DEFENSE_RADIUS) ab_attack(S, L, w.uid, e.uid);
            else harvest_behavior(S, L, w);
        }
    }
}

// ---- lane-parallel behaviours (the rush family and coacAI, <= 64 units) --------
// The behaviours above visit the player's units one after another, each decision
// a chain of wave-wide steps.  No decision reads another unit's decision: a unit
// reads the fixed state and only its own abstract action, and at most one
// behaviour puts an entry for it in a tick.  So every unit decides in its own
// lane at once, and the puts are then applied as the serial loops would: an
// existing key is replaced in place, new keys are appended in visiting order
// (bases, barracks, army, workers; pgs.units order within each).  Only the at
// most two building workers (findBuildingPosition + its reservations) decide
// serially, before the rest.  Bit-identical to the serial behaviours (and so
// to the oracle); used while the unit list and the abstract-action list fit a
// wave.
struct LaneDecision {
    int cat;       // visiting category of the put: 0 bases, 1 barracks, 2 army, 3 workers; -1 = no put
    int4 a, b;     // the entry put
    bool explore;  // PO* exploration: target decided afterwards (serially: a full-map scan each)
};
__device__ __forceinline__ int lane_gather(int v, int src) { return __shfl(v, src); }   // per-lane source lane

// the player's units that are stockpiles / resources, nearest to this lane's unit (list index, -1 none)
__device__ __forceinline__ int lane_closest(const BS& S, unsigned long long cand) {
    const int ux = S.kcell % S.W, uy = S.kcell / S.W;
    uint32_t key = 0xFFFFFFFFu;
    while (cand) {
        const int j = __builtin_ctzll(cand);
        cand &= cand - 1ull;
        const int c = lane_value(S.kcell, j);
        const uint32_t kk = ((uint32_t)(iabs(c % S.W - ux) + iabs(c / S.W - uy)) << 16) | (uint32_t)j;
        key = kk < key ? kk : key;
    }
    return key == 0xFFFFFFFFu ? -1 : (int)(key & 0xFFFFu);
}

// army: 0 = coacAI (its own worker / army rules), else the rush's army unit type
__device__ __forceinline__ void behaviours_parallel(BS& S, const BL& L, int army, bool po, bool coac) {
    const int lane = blane(), p = S.player, res = p ? S.res[1] : S.res[0];
    const bool valid = lane < S.n;
    const uint32_t u = S.kunit;
    const int t = u_type(u), ow = u_owner(u);
    const bool own = valid && ow == p, idle = own && S.kact == 0;
    const unsigned long long own_workers = __ballot(own && ut_can_harvest(t));
    const int nworkers = __popcll(__ballot(own && t == WORKER)), nbases = __popcll(__ballot(own && t == BASE)),
              nbarracks = __popcll(__ballot(own && t == BARRACKS)), nf = __popcll(own_workers);
    // this lane's existing abstract action (keys are unique): its index from one
    // scalar read per entry, then the entry itself gathered from that lane
    int ek = -1;
    for (int j = 0; j < S.naa; j++)   // (lane reads outside the divergent branch)
        if (ek < 0 && lane_value(S.kA.x, j) == S.kuid) ek = j;
    if (!own) ek = -1;
    const int es = max(ek, 0);
    int4 ea = make_int4(lane_gather(S.kA.x, es), lane_gather(S.kA.y, es), lane_gather(S.kA.z, es), lane_gather(S.kA.w, es));
    int4 eb = make_int4(lane_gather(S.kB.x, es), lane_gather(S.kB.y, es), lane_gather(S.kB.z, es), lane_gather(S.kB.w, es));
    if (ek < 0) {
        ea = make_int4(0, 0, 0, 0);
        eb = make_int4(0, 0, 0, 0);
    }
    LaneDecision d{-1, make_int4(0, 0, 0, 0), make_int4(-1, 0, 0, 0), false};
    const int rank = __popcll(own_workers & ((1ull << lane) - 1ull));   // position among the player's workers
    // builders (serial): base first, then (not WorkerRush) barracks
    Rsv reserved{0, 0, 0};
    int used = 0, head = 0;
    auto build = [&](int type) {
        const int k = nth_index(S, L, head, [&](int, uint32_t uu, uint32_t) { return ut_can_harvest(u_type(uu)) && u_owner(uu) == p; });
        const URef w = ref_at(S, L, k);
        const int e = find_aa(S, L, w.uid);
        bool skip = false;
        if (e >= 0) {
            int4 a0, b0;
            aa_entry(S, L, e, a0, b0);
            skip = aa_kind(a0) == AA_BUILD && aa_utype(a0) == type;
        }
        if (!skip) {
            const int pos = find_building_position(S, L, reserved, w.c % S.W, w.c / S.W);
            if (lane == k) {
                d.cat = 3;
                d.a = make_int4(w.uid, AA_BUILD | (type << 4), -1, pk_xy(pos % S.W, pos / S.W));   // Java division: -1 -> (-1, 0)
                d.b = make_int4(-1, 0, 0, 0);
            }
            if (reserved.n == 0) reserved.a = pos;
            else reserved.b = pos;
            reserved.n++;
        }
        head++;
    };
    if (nf > 0 && nbases == 0 && res >= ut_cost(BASE)) {
        build(BASE);
        used += ut_cost(BASE);
    }
    if (army != WORKER && nf > head && nbarracks == 0 && res >= ut_cost(BARRACKS) + used &&
        (!coac || nworkers >= COAC_BARRACKS_MIN_WORKERS)) {
        build(BARRACKS);
        used += ut_cost(BARRACKS);
    }
    // every other unit in its lane
    const int tarmy = coac ? (__popcll(__ballot(valid && ow >= 0 && ow != p && t == LIGHT)) >
                                      __popcll(__ballot(valid && ow >= 0 && ow != p && t == RANGED)) +
                                          __popcll(__ballot(valid && ow >= 0 && ow != p && t == HEAVY))
                                  ? HEAVY : RANGED)
                           : army;
    const bool base_train = coac ? (nworkers < COAC_HARVESTERS_PER_BASE * nbases + COAC_EXTRA_WORKERS && res >= ut_cost(WORKER))
                                 : (army == WORKER ? res >= ut_cost(WORKER) : nworkers < 1 && res >= ut_cost(WORKER));
    const int enemy = S.kenemy;
    const int enemy_uid = lane_gather(S.kuid, max(enemy, 0));
    const int enemy_cell = lane_gather(S.kcell, max(enemy, 0));
    const unsigned long long resources = __ballot(valid && t == RESOURCE), stockpiles = __ballot(own && ut_is_stockpile(t));
    int ri = -1, bi = -1;
    if (own && ut_can_harvest(t)) {
        ri = lane_closest(S, resources);
        bi = lane_closest(S, stockpiles);
    }
    const int r_uid = lane_gather(S.kuid, max(ri, 0)), b_uid = lane_gather(S.kuid, max(bi, 0)), b_cell = lane_gather(S.kcell, max(bi, 0));
    auto harvest = [&]() {
        if (ri < 0 || bi < 0) return;
        if (ek >= 0 && aa_kind(ea) == AA_HARVEST && ea.z == r_uid && eb.x == b_uid) return;
        d.cat = 3;
        d.a = make_int4(S.kuid, AA_HARVEST, r_uid, 0);
        d.b = make_int4(b_uid, pk_xy(b_cell % S.W, b_cell / S.W), 0, 0);
    };
    auto melee = [&](int cat) {
        if (enemy >= 0) {
            d.cat = cat;
            d.a = make_int4(S.kuid, AA_ATTACK, enemy_uid, 0);
            d.b = make_int4(-1, 0, 0, 0);
        } else if (po && S.partial) {
            d.cat = cat;
            d.explore = true;
        }
    };
    if (idle && t == BASE) {
        if (base_train) {
            d.cat = 0;
            d.a = make_int4(S.kuid, AA_TRAIN | (WORKER << 4), -1, 0);
        }
    } else if (idle && t == BARRACKS) {
        if (army != WORKER && res >= ut_cost(tarmy)) {
            d.cat = 1;
            d.a = make_int4(S.kuid, AA_TRAIN | (tarmy << 4), -1, 0);
        }
    } else if (idle && ut_can_attack(t) && !ut_can_harvest(t)) {
        melee(2);
    } else if (own && ut_can_harvest(t) && rank >= head) {
        if (coac) {
            const int nh = COAC_HARVESTERS_PER_BASE * (nbases > 0 ? nbases : 1);
            if (rank - head < nh) {
                harvest();
            } else if (enemy >= 0) {   // defenders
                if (bi < 0 || iabs(b_cell % S.W - enemy_cell % S.W) + iabs(b_cell / S.W - enemy_cell / S.W) <= COAC_DEFENSE_RADIUS) {
                    d.cat = 3;
                    d.a = make_int4(S.kuid, AA_ATTACK, enemy_uid, 0);
                    d.b = make_int4(-1, 0, 0, 0);
                } else {
                    harvest();
                }
            }
        } else if (army == WORKER) {
            if (rank == head) harvest();
            else melee(3);
        } else {
            harvest();
        }
    }
    // PO* exploration targets: the nearest cell the player cannot observe (row-major first)
    unsigned long long ex = __ballot(d.explore);
    while (ex) {
        const int j = __builtin_ctzll(ex);
        ex &= ex - 1ull;
        const int cj = lane_value(S.kcell, j), ux = cj % S.W, uy = cj / S.W;
        uint32_t key = 0xFFFFFFFFu;
        for (int c = lane; c < S.HW; c += BT) {
            if (bit_at(L.vis, c)) continue;
            const int x = c % S.W, y = c / S.W;
            const uint32_t kk = ((uint32_t)((ux - x) * (ux - x) + (uy - y) * (uy - y)) << 16) | (uint32_t)c;
            key = kk < key ? kk : key;
        }
        key = wave_min_u32(key);
        if (lane == j) {
            if (key == 0xFFFFFFFFu) {
                d.cat = -1;
            } else {
                const int c = (int)(key & 0xFFFFu);
                d.a = make_int4(S.kuid, AA_MOVE, -1, pk_xy(c % S.W, c / S.W));
                d.b = make_int4(-1, 0, 0, 0);
            }
        }
    }
    // apply the puts: replace in place, append new keys in visiting order
    const bool put = d.cat >= 0, fresh = put && ek < 0;
    int pos = ek, appended = 0;
    for (int cat = 0; cat < 4; cat++) {
        const unsigned long long m = __ballot(fresh && d.cat == cat);
        if (fresh && d.cat == cat) pos = S.naa + appended + __popcll(m & ((1ull << lane) - 1ull));
        appended += __popcll(m);
    }
    if (S.naa + appended > S.HW) {   // more live entries than cells: cannot happen on legal states
        if (lane0()) L.sc[2] |= MRTS_ERR_BOT_OVERFLOW;
        return;
    }
    if (put) {
        L.aa[2 * pos] = d.a;
        L.aa[2 * pos + 1] = d.b;
    }
    S.naa += appended;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (S.naa <= BT) {
        S.kA = lane < S.naa ? L.aa[2 * lane] : make_int4((int)0x80000000, 0, 0, 0);
        S.kB = lane < S.naa ? L.aa[2 * lane + 1] : make_int4(0, 0, 0, 0);
    }
}

// ---- RandomBiasedAI ------------------------------------------------------------------
__device__ __forceinline__ void philox_b(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Unit.getUnitActions(gs, 10) enumerated in order on the bot's view.  Calls
// f(code, weight) per action (weight 5 for attack / harvest / return).
template <typename F>
__device__ __forceinline__ void unit_actions(const BS& S, const BL& L, int c, F f) {
    const Grid gd{S.W, S.H, S.HW};
    const uint32_t u = L.unit[c];
    const int t = u_type(u), me = u_owner(u), ux = c % S.W, uy = c / S.W;
    int nb[4];
    for (int d = 0; d < 4; d++) nb[d] = nb_cell(gd, c, d);
    const int A = MRTS_ATTACK_GRID / 2;
    if (ut_can_attack(t)) {
        if (ut_range(t) == 1) {
            for (int d = 0; d < 4; d++) {
                if (nb[d] < 0 || L.unit[nb[d]] == 0) continue;
                const int o = u_owner(L.unit[nb[d]]);
                if (o != me && o >= 0) f(code_make(A_ATTACK, (dir_dy(d) + A) * MRTS_ATTACK_GRID + dir_dx(d) + A, 0), 5);
            }
        } else {
            const int r2 = ut_range(t) * ut_range(t);
            for (int k = 0; k < S.n; k++) {
                const int oc = L.ucell[k];
                const int o = u_owner(L.unit[oc]);
                if (o < 0 || o == me) continue;
                const int dx = oc % S.W - ux, dy = oc / S.W - uy;
                if (dx * dx + dy * dy <= r2) f(code_make(A_ATTACK, (dy + A) * MRTS_ATTACK_GRID + dx + A, 0), 5);
            }
        }
    }
    if (ut_can_harvest(t)) {
        if (u_res(u) == 0)
            for (int d = 0; d < 4; d++)
                if (nb[d] >= 0 && L.unit[nb[d]] != 0 && u_type(L.unit[nb[d]]) == RESOURCE) f(code_make(A_HARVEST, d, 0), 5);
        if (u_res(u) > 0)
            for (int d = 0; d < 4; d++)
                if (nb[d] >= 0 && L.unit[nb[d]] != 0 && ut_is_stockpile(u_type(L.unit[nb[d]])) && u_owner(L.unit[nb[d]]) == me)
                    f(code_make(A_RETURN, d, 0), 5);
    }
    const int prod = ut_produces(t);
    for (int pt = 0; pt < MRTS_NTYPES; pt++) {
        if (!((prod >> pt) & 1) || (me ? S.res[1] : S.res[0]) < ut_cost(pt)) continue;
        for (int d = 0; d < 4; d++)
            if (nb[d] >= 0 && !L.wall[nb[d]] && L.unit[nb[d]] == 0) f(code_make(A_PRODUCE, d, pt), 1);
    }
    if (ut_can_move(t))
        for (int d = 0; d < 4; d++)
            if (nb[d] >= 0 && !L.wall[nb[d]] && L.unit[nb[d]] == 0) f(code_make(A_MOVE, d, 0), 1);
    f(code_make(A_NONE, 10, 0), 1);
}

__device__ __forceinline__ void random_biased_get_action(BS& S, const BL& L) {
    // pa.ru starts as the usage of every pending assignment
    S.pa_res[0] = S.pend_res[0];
    S.pa_res[1] = S.pend_res[1];
    const int posw = (S.HW + 2 * S.W) / 32 + 1;
    for (int i = blane(); i < posw; i += BT) L.pab[i] = L.pend[i];
    for_each_unit(S, L, [&](int, uint32_t u, uint32_t a) { return u_owner(u) == S.player && a == 0; }, [&](const URef& ur) {
        const int c = ur.c;
        int total = 0;
        unit_actions(S, L, c, [&](int, int w) { total += w; });
        uint32_t ctr[4] = {(uint32_t)ur.uid, S.tick, (uint32_t)S.game, 0x52414E44u + (uint32_t)(1 - S.player)};
        philox_b(ctr, 0x5EED5EEDu, 0xB0B0B0B0u);
        int t = (int)(((uint64_t)ctr[0] * (uint32_t)total) >> 32), pick = -1;
        unit_actions(S, L, c, [&](int code, int w) {
            if (pick < 0) {
                t -= w;
                if (t < 0) pick = code;
            }
        });
        if (pick < 0) pick = code_make(A_NONE, 10, 0);
        RU r = usage(S, c, pick, S.player);
        if (consistent(S, r, L.pab, S.pa_res)) pa_add(S, L, c, pick);
        else pa_add(S, L, c, code_make(A_NONE, 10, 0));
    });
}


// RandomBiasedSingleUnitAI (randomAI): one unit acts at a time (oracle
// random_single_get_action): nothing while a unit of the player is busy, else
// one idle unit drawn uniformly gets a RandomBiasedAI-weighted action
__device__ __forceinline__ void random_single_get_action(BS& S, const BL& L) {
    auto own = [&](int, uint32_t u, uint32_t) { return u_owner(u) == S.player; };
    if (count_where(S, L, [&](int, uint32_t u, uint32_t a) { return u_owner(u) == S.player && a != 0; }) > 0) return;
    const int ni = count_where(S, L, own);
    if (ni == 0) return;
    S.pa_res[0] = S.pend_res[0];
    S.pa_res[1] = S.pend_res[1];
    const int posw = (S.HW + 2 * S.W) / 32 + 1;
    for (int i = blane(); i < posw; i += BT) L.pab[i] = L.pend[i];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    uint32_t ctr[4] = {0xFFFFFFFFu, S.tick, (uint32_t)S.game, 0x52534E47u + (uint32_t)(1 - S.player)};
    philox_b(ctr, 0x5EED5EEDu, 0xB0B0B0B0u);
    const int c = ref_at(S, L, nth_index(S, L, (int)(((uint64_t)ctr[1] * (uint32_t)ni) >> 32), own)).c;
    int total = 0;
    unit_actions(S, L, c, [&](int, int w) { total += w; });
    int t = (int)(((uint64_t)ctr[0] * (uint32_t)total) >> 32), pick = -1;
    unit_actions(S, L, c, [&](int code, int w) {
        if (pick < 0) {
            t -= w;
            if (t < 0) pick = code;
        }
    });
    if (pick < 0) pick = code_make(A_NONE, 10, 0);
    RU r = usage(S, c, pick, S.player);
    pa_add(S, L, c, consistent(S, r, L.pab, S.pa_res) ? pick : code_make(A_NONE, 10, 0));
}

// workgroup barrier of the one-wave k_bot; inside k_step only wave 0 runs the
// bot, so a wave-level LDS fence (a single wave's LDS operations complete in order)
template <bool FUSED>
__device__ __forceinline__ void bot_sync() {
    if (FUSED) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}


// ---- the kernel ------------------------------------------------------------------------
// ai.getAction(player, gs) of bot game b, by ONE wavefront (lanes = blane()
// 0..63), LDS at `smem` (bot_lds_bytes).  FUSED: run by wave 0 of a k_step
// workgroup for the NEXT tick while the other waves stream the outputs (no
// workgroup barriers here then; the game state was stored before the caller's
// last barrier); otherwise the body of k_bot (a one-wave workgroup).
// FUSED: `tail` (the small arrays' region) and `step_wall` (the step's terrain,
// read in place) are the fused k_step layout's (mrts_engine.hip fb_*_offset).

template <bool FUSED>
__device__ __forceinline__ void bot_game(const EngineParams& p, int b, int player, unsigned char* smem,
                                         const int32_t* step_sc = nullptr, bool pre_ok = false, int4 pre_aa = int4{0, 0, 0, 0},
                                         int4 pre_aa2 = int4{0, 0, 0, 0}, unsigned char* tail = nullptr,
                                         const uint8_t* step_wall = nullptr, bool preset = false) {
    const int g = p.nsp_games + b, lane = blane();
    const int HW = p.HW, W = p.W;
    int32_t* genv = p.genv + (size_t)g * MRTS_GENV_WORDS;
    const int w_aa = player ? MRTS_G_AA_N : MRTS_G_AA_N0, w_npa = player ? MRTS_G_NPA : MRTS_G_NPA0;
    BS S;
#ifdef MRTS_STAMPS
    S.c_entries = S.c_searches = S.c_ticks = S.c_rounds = 0;
#endif
    S.ai = player ? p.bot_ai[b] : (p.bot_ai0 ? p.bot_ai0[b] : -1);
    if (S.ai < 0) return;            // the agent plays this side
    if (S.ai == MRTS_AI_PASSIVE) {   // PassiveAI: all NONE (k_step's fill)
        if (lane0()) genv[w_npa] = 0;
        return;
    }
    BL L = bot_carve(smem, HW, W, tail, step_wall == nullptr);
    // the fused bot reads the step's terrain in place (the waves beside it read it too)
    if (step_wall) L.wall = const_cast<uint8_t*>(step_wall);
    int4* const aa_g = p.aa + ((size_t)b * 2 + player) * HW * 2;
    int32_t* const pa_g = p.botpa + ((size_t)b * 2 + player) * HW;
    S.W = W;
    S.H = p.H;
    S.HW = HW;
    S.player = player;
    S.partial = p.partial_obs;
    S.game = p.game_offset + g;
    // the game's scalars: the step kernel's LDS copy when fused (read before the
    // bot's first LDS write), else the stored genv
    const int32_t* gs = FUSED ? step_sc : genv;
    S.tick = (uint32_t)gs[MRTS_G_TICKS];
    S.res[0] = gs[MRTS_G_RES0];
    S.res[1] = gs[MRTS_G_RES1];
    S.naa = gs[w_aa];
    S.npa = 0;
    S.pa_res[0] = S.pa_res[1] = 0;
    const int map = gs[MRTS_G_MAP];
    const int posw = (HW + 2 * W) / 32 + 1, visw = HW / 32 + 1;
    // Fused: the step kernel's unit / uid / act arrays sit at the bot's offsets
    // (both carves start unit, uid, act of 4*HW bytes at smem 0) and hold the
    // state it has just stored -- no reload.
    // Fused, the first 128 abstract-action words come prefetched in registers
    // (pre_aa / pre_aa2: words lane, lane + 64).
    // preset (the fused k_step's early bot, full observability): the workgroup has
    // already built the pending reservations, the free-cell words and the unit list
    // (mrts_engine.hip bot_setup_workgroup) and zeroed the tail arrays
    for (int c = lane; !preset && c < HW; c += BT) {
        if (!FUSED) {
            int4 v = p.cells[(size_t)g * p.cstride + c];
            L.unit[c] = (uint32_t)v.x;
            L.uid[c] = v.y;
            L.act[c] = (uint32_t)v.z;
        }
        if (!step_wall) L.wall[c] = p.map_wall[(size_t)map * HW + c];
    }
    for (int i = lane; !preset && i < posw; i += BT) L.pend[i] = L.pab[i] = 0;
    for (int i = lane; !preset && i < visw; i += BT) L.vis[i] = 0;
    {   // the abstract actions: the first 128 words come prefetched in registers when fused
        int i0 = 0;
        if (FUSED && pre_ok) {   // no global load is issued for them
            if (lane < 2 * S.naa) L.aa[lane] = pre_aa;
            if (BT + lane < 2 * S.naa) L.aa[BT + lane] = pre_aa2;
            i0 = 2 * BT;
        }
        for (int i = i0 + lane; i < 2 * S.naa; i += BT) L.aa[i] = aa_g[i];
    }
    if (!preset && lane < 3) L.sc[lane] = 0;   // pending produce cost per player, error bits
    bot_sync<FUSED>();
    // cells observable by the bot's player (PartiallyObservableGameState);
    // read only under partial observability (hidden units, PO* exploration)
    for (int c = lane; S.partial && c < HW; c += BT) {
        const uint32_t u = L.unit[c];
        if (u == 0 || u_owner(u) != S.player) continue;
        or_sight_disk(L.vis, c % W, c / W, ut_sight(u_type(u)), W, p.H);
    }
    bot_sync<FUSED>();
    if (S.partial) {   // hide the units the player cannot observe
        for (int c = lane; c < HW; c += BT) {
            const uint32_t u = L.unit[c];
            if (u != 0 && u_owner(u) != S.player && !bit_at(L.vis, c)) {
                L.unit[c] = 0;
                L.act[c] = 0;
            }
        }
        bot_sync<FUSED>();
    }
    // pending reservations of the visible units (isUnitActionAllowed)
    for (int c = lane; !preset && c < HW; c += BT) {
        const uint32_t a = L.act[c];
        if (a == 0) continue;
        const int code = act_code(a), t = code_type(code);
        if (t != A_MOVE && t != A_PRODUCE) continue;
        RU r = usage(S, c, code, u_owner(L.unit[c]));
        atomicOr(&L.pend[(r.pos + W) >> 5], 1u << ((r.pos + W) & 31));
        if (t == A_PRODUCE) atomicAdd(&L.sc[u_owner(L.unit[c])], u_owner(L.unit[c]) ? r.res[1] : r.res[0]);
    }
    // units in pgs.units order: ordered compaction by cell, then rank by uid
    int n = preset ? L.sc[3] : 0;
    for (int base = 0; !preset && base < HW; base += BT) {
        const int c = base + lane;
        const bool has = c < HW && L.unit[c] != 0;
        const unsigned long long m = __ballot(has);
        if (has) L.pa[n + __popcll(m & ((1ull << lane) - 1ull))] = c;
        n += __popcll(m);
    }
    bot_sync<FUSED>();
    if (preset) {
    } else if (n <= BT) {   // rank by uid with the uids in registers (one per lane)
        const int c = lane < n ? L.pa[lane] : 0, u = lane < n ? L.uid[c] : 0x7fffffff;
        int r = 0;
        for (int j = 0; j < n; j++) r += lane_value(u, j) < u;
        if (lane < n) {
            L.ucell[r] = c;
            L.uuid[r] = u;
        }
    } else {
        for (int i = lane; i < n; i += BT) {
            const int c = L.pa[i], u = L.uid[c];
            int r = 0;
            for (int j = 0; j < n; j++) r += L.uid[L.pa[j]] < u;
            L.ucell[r] = c;
            L.uuid[r] = u;
        }
    }
    bot_sync<FUSED>();
    S.n = n;
    S.kcell = lane < n ? L.ucell[lane] : 0;   // the list in registers (used while n <= 64)
    S.kuid = lane < n ? L.uuid[lane] : (int)0x80000000;
    S.kunit = lane < n ? L.unit[S.kcell] : 0u;
    S.kact = lane < n ? L.act[S.kcell] : 0u;
    S.kA = lane < S.naa ? L.aa[2 * lane] : make_int4((int)0x80000000, 0, 0, 0);
    S.kB = lane < S.naa ? L.aa[2 * lane + 1] : make_int4(0, 0, 0, 0);
    S.pend_res[0] = L.sc[0];
    S.pend_res[1] = L.sc[1];
    // lane y: free cells of row y, from one ballot per 64 cells (staged in L.pa,
    // free until the PlayerAction is built)
    S.rurow = 0;
    {
        uint32_t* fw = L.fw;
        const int nwords = (HW + 63) / 64 * 2;
        for (int base = 0; !preset && base < HW; base += BT) {
            const int c = base + lane;
            const unsigned long long m = __ballot(c < HW && !L.wall[c] && L.unit[c] == 0);
            if (lane == 0) {
                fw[base / 32] = (uint32_t)m;
                fw[base / 32 + 1] = (uint32_t)(m >> 32);
            }
        }
        if (!preset && lane == 0) fw[nwords] = 0u;   // the row window's upper word past the last cell
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        S.frow = 0;
        if (lane < p.H) {
            const int o = lane * W, q = o >> 5;
            const uint64_t win = ((uint64_t)fw[q + 1] << 32) | fw[q];
            S.frow = (uint32_t)(win >> (o & 31)) & (W == 32 ? 0xFFFFFFFFu : ((1u << W) - 1u));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    // the closest enemy (list index) of each of the player's units, the scan
    // closest_enemy_index would do, all units at once (the state is fixed during
    // getAction): in lane k's kenemy, or L.pa[k] past 64 units; -1 = none
    if (FUSED) MRTS_STAMP(10, lane == 0);
    const bool table = S.ai != MRTS_AI_RANDOM_BIASED && S.ai != MRTS_AI_RANDOM;
    S.kenemy = -1;
    if (table && n <= BT) {   // over the opponent's units only (scalar lane reads of their cells)
        const int ux = S.kcell % W, uy = S.kcell / W;
        uint32_t key = 0xFFFFFFFFu;
        unsigned long long m = __ballot(lane < n && u_owner(S.kunit) == 1 - S.player);
        while (m) {
            const int j = __builtin_ctzll(m);
            m &= m - 1ull;
            const int c = lane_value(S.kcell, j);
            const uint32_t kk = ((uint32_t)(iabs(c % W - ux) + iabs(c / W - uy)) << 16) | (uint32_t)j;
            key = kk < key ? kk : key;
        }
        if (lane < n && u_owner(S.kunit) == S.player && key != 0xFFFFFFFFu) S.kenemy = (int)(key & 0xFFFFu);
    }
    for (int k = lane; table && n > BT && k < n; k += BT) {
        const int cu = L.ucell[k], me = u_owner(L.unit[cu]), ux = cu % W, uy = cu / W;
        uint32_t key = 0xFFFFFFFFu;
        for (int j = 0; me == S.player && j < n; j++) {
            const int c = L.ucell[j];
            const int o = u_owner(L.unit[c]);
            if (o < 0 || o == me) continue;
            const uint32_t kk = ((uint32_t)(iabs(c % W - ux) + iabs(c / W - uy)) << 16) | (uint32_t)j;
            key = kk < key ? kk : key;
        }
        L.pa[k] = key == 0xFFFFFFFFu ? -1 : (int)(key & 0xFFFFu);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // getAction: the rush family and coacAI decide their abstract actions (lane-
    // parallel while the unit list and the action list fit a wave, else unit by unit)
    // and translate them; one call site per routine, with the AI's parameters as
    // values -- per-AI constant copies made the inlined bot several times larger
    // (an instruction-cache cost for the latency-bound bot wave)
    const bool coac = S.ai == MRTS_AI_COAC;
    int army = -1;
    bool po = false;
    switch (S.ai) {
    case MRTS_AI_WORKER_RUSH: army = WORKER; break;
    case MRTS_AI_LIGHT_RUSH: army = LIGHT; break;
    case MRTS_AI_PO_WORKER_RUSH: army = WORKER; po = true; break;
    case MRTS_AI_PO_LIGHT_RUSH: army = LIGHT; po = true; break;
    case MRTS_AI_PO_HEAVY_RUSH: army = HEAVY; po = true; break;
    case MRTS_AI_PO_RANGED_RUSH: army = RANGED; po = true; break;
    default: break;
    }
    if (coac || army >= 0) {
        if (S.n <= BT && S.naa <= BT) behaviours_parallel(S, L, coac ? 0 : army, po, coac);
        else if (coac) coac_serial(S, L);
        else rush_serial(S, L, army, po);
        if (FUSED) MRTS_STAMP(11, lane == 0);
        translate_actions(S, L);
    } else if (S.ai == MRTS_AI_RANDOM_BIASED) {
        random_biased_get_action(S, L);
    } else if (S.ai == MRTS_AI_RANDOM) {
        random_single_get_action(S, L);
    }
    bot_sync<FUSED>();
    if (FUSED) MRTS_STAMP(12, lane == 0);
    MRTS_STAMP_ADD(16, S.c_entries, FUSED && lane == 0);
    MRTS_STAMP_ADD(17, S.c_searches, FUSED && lane == 0);
    MRTS_STAMP_ADD(18, S.c_ticks, FUSED && lane == 0);
    MRTS_STAMP_ADD(19, S.c_rounds, FUSED && lane == 0);
    for (int i = lane; i < S.npa; i += BT) pa_g[i] = L.pa[i];
    for (int i = lane; i < 2 * S.naa; i += BT) aa_g[i] = L.aa[i];
    if (lane0()) {
        genv[w_npa] = S.npa;
        genv[w_aa] = S.naa;
        if (L.sc[2]) atomicOr(&genv[MRTS_G_ERR], L.sc[2]);
    }
}


}  // namespace bots
}  // namespace mrts
#endif
