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
    int* sc;
};

__host__ __device__ inline size_t b16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t bot_lds_bytes(int HW, int W) {
    const size_t posw = (size_t)(HW + 2 * W) / 32 + 1;
    return b16(4 * (size_t)HW) * 6 + b16(32 * (size_t)HW) + 2 * b16(4 * posw) + b16(4 * ((size_t)HW / 32 + 1)) +
           b16((size_t)HW) + b16(4 * 32);
}

__device__ __forceinline__ BL bot_carve(unsigned char* base, int HW, int W) {
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
    L.pend = (uint32_t*)take(4 * posw);
    L.pab = (uint32_t*)take(4 * posw);
    L.vis = (uint32_t*)take(4 * ((size_t)HW / 32 + 1));
    L.wall = (uint8_t*)take((size_t)HW);
    L.sc = (int*)take(4 * 32);
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
};

__device__ __forceinline__ bool lane0() { return threadIdx.x == 0; }
__device__ __forceinline__ int iabs(int a) { return a < 0 ? -a : a; }

__device__ __forceinline__ bool in_map(const BS& S, int x, int y) { return x >= 0 && y >= 0 && x < S.W && y < S.H; }
__device__ __forceinline__ bool v_free(const BS& S, const BL& L, int x, int y) {   // GameState.free
    if (!in_map(S, x, y)) return false;
    int c = y * S.W + x;
    return !L.wall[c] && L.unit[c] == 0;
}

// uid -> cell in the bot's view (binary search over the uid-ordered list), -1 if absent
__device__ __forceinline__ int cell_of_uid(const BS& S, const BL& L, int uid) {
    int lo = 0, hi = S.n - 1;
    while (lo <= hi) {
        int mid = (lo + hi) >> 1, v = L.uuid[mid];
        if (v == uid) return L.ucell[mid];
        if (v < uid) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// ---- wave-parallel scans of the unit list (results identical in every lane) ----
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long k) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(k, o);
        k = v < k ? v : k;
    }
    return k;
}
// The first unit in pgs.units order (a serial `d < best` scan) among those
// `want` selects minimising the Manhattan distance to (x, y): min over
// (distance, list index) across the lanes.  -1 if none; *dist = that distance.
template <typename F>
__device__ __forceinline__ int closest_unit(const BS& S, const BL& L, int x, int y, F want, int* dist = nullptr) {
    unsigned long long key = ~0ull;
    for (int k = threadIdx.x; k < S.n; k += BT) {
        const int c = L.ucell[k];
        if (!want(c)) continue;
        const unsigned d = (unsigned)(iabs(c % S.W - x) + iabs(c / S.W - y));
        const unsigned long long kk = ((unsigned long long)d << 32) | (unsigned)k;
        key = kk < key ? kk : key;
    }
    key = wave_min_u64(key);
    if (key == ~0ull) return -1;
    if (dist) *dist = (int)(key >> 32);
    return L.ucell[(int)(key & 0xFFFFFFFFu)];
}
// number of units `want` selects
template <typename F>
__device__ __forceinline__ int count_where(const BS& S, const BL& L, F want) {
    int n = 0;
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + threadIdx.x;
        n += __popcll(__ballot(k < S.n && want(L.ucell[k])));
    }
    return n;
}
// the idx-th unit (pgs.units order) `want` selects, -1 if fewer
template <typename F>
__device__ __forceinline__ int nth_where(const BS& S, const BL& L, int idx, F want) {
    for (int base = 0; base < S.n; base += BT) {
        const int k = base + threadIdx.x;
        unsigned long long m = __ballot(k < S.n && want(L.ucell[k]));
        const int cnt = __popcll(m);
        if (idx < cnt) {
            for (int t = 0; t < idx; t++) m &= m - 1ull;
            return L.ucell[base + __builtin_ctzll(m)];
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
    if (r.pos != -0x7fffffff && r.pos >= 0 && r.pos < S.HW && (int)threadIdx.x == r.pos / S.W)
        S.rurow |= 1u << (r.pos % S.W);
}

// ---- AStarPathFinding.findPathToPositionInRange (restated: DESIGN.md §4b) ----
// Breadth-first layers grow from the goal set (free cells within `range` of
// the target) over free cells; the first layer that touches a free neighbour
// of the start decides the move, ties UP, RIGHT, DOWN, LEFT.  -1 = null.
__device__ __forceinline__ int pf_dir(const BS& S, int sc, int tx, int ty, int range) {
    const int lane = threadIdx.x, sx = sc % S.W, sy = sc / S.W, r2 = range * range;
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
    uint32_t seen = goal, front = goal;
    for (int it = 0; it <= S.HW; it++) {
        const uint32_t rU = __shfl(front, max(sy - 1, 0)), rC = __shfl(front, sy), rD = __shfl(front, min(sy + 1, 63));
        if (sy > 0 && ((rU >> sx) & 1u)) return 0;
        if (sx + 1 < S.W && ((rC >> (sx + 1)) & 1u)) return 1;
        if (sy + 1 < S.H && ((rD >> sx) & 1u)) return 2;
        if (sx > 0 && ((rC >> (sx - 1)) & 1u)) return 3;
        uint32_t up = __shfl_up(front, 1), dn = __shfl_down(front, 1);
        if (lane == 0) up = 0;
        if (lane >= S.H - 1) dn = 0;
        const uint32_t grow = ((front << 1) | (front >> 1) | up | dn) & rowmask & fr & ~seen;
        seen |= grow;
        front = grow;
        if (!__any(grow != 0)) return -1;
    }
    return -1;
}

// ---- abstract actions ----------------------------------------------------------
__device__ __forceinline__ int find_aa(const BS& S, const BL& L, int uid) {   // first entry of the unit, lane-parallel
    for (int base = 0; base < S.naa; base += BT) {
        const int k = base + threadIdx.x;
        const unsigned long long m = __ballot(k < S.naa && L.aa[2 * k].x == uid);
        if (m) return base + __builtin_ctzll(m);
    }
    return -1;
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
    closest_unit(S, L, x, y, [&](int c) {
        const uint32_t o = L.unit[c];
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
__device__ __forceinline__ void translate_actions(BS& S, const BL& L) {
    int w = 0;
    const int n0 = S.naa;
    for (int k = 0; k < n0; k++) {
        int4 a = L.aa[2 * k];
        const int4 b = L.aa[2 * k + 1];
        const int cu = cell_of_uid(S, L, a.x);
        const bool del = cu < 0 || aa_completed(S, L, a, cu);
        if (!del && L.act[cu] == 0) {
            const int code = aa_execute(S, L, a, b, cu);
            if (code >= 0) {
                RU r = usage(S, cu, code, u_owner(L.unit[cu]));
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
    S.naa = w;
}

// ---- behaviours ------------------------------------------------------------------
// closest enemy of the unit at cu: precomputed for every unit in k_bot before
// the behaviours (L.pa[cell]) for the rush family; wave-parallel scan otherwise
__device__ __forceinline__ int closest_enemy(const BS& S, const BL& L, int cu, bool table = true) {
    if (table) return L.pa[cu];
    const int me = u_owner(L.unit[cu]);
    return closest_unit(S, L, cu % S.W, cu / S.W, [&](int c) {
        const int o = u_owner(L.unit[c]);
        return o >= 0 && o != me;
    });
}
__device__ __forceinline__ int closest_of(const BS& S, const BL& L, int cu, bool want_resource) {
    const int me = u_owner(L.unit[cu]);
    return closest_unit(S, L, cu % S.W, cu / S.W, [&](int c) {
        const uint32_t o = L.unit[c];
        return want_resource ? u_type(o) == RESOURCE : (ut_is_stockpile(u_type(o)) && u_owner(o) == me);
    });
}

// meleeUnitBehavior (+ PO* exploration: nearest cell the player cannot observe)
__device__ __forceinline__ void melee_behavior(BS& S, const BL& L, int cu, bool po) {
    const int e = closest_enemy(S, L, cu);
    if (e >= 0) {
        ab_attack(S, L, L.uid[cu], L.uid[e]);
        return;
    }
    if (!(po && S.partial)) return;
    const int ux = cu % S.W, uy = cu / S.W;
    // first minimum in row-major scan order = min over (d^2, cell)
    unsigned long long key = ~0ull;
    for (int c = threadIdx.x; c < S.HW; c += BT) {
        if (bit_at(L.vis, c)) continue;
        const int x = c % S.W, y = c / S.W;
        const unsigned long long kk = ((unsigned long long)((ux - x) * (ux - x) + (uy - y) * (uy - y)) << 32) | (unsigned)c;
        key = kk < key ? kk : key;
    }
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long v = __shfl_xor(key, o);
        key = v < key ? v : key;
    }
    if (key != ~0ull) {
        const int c = (int)(key & 0xFFFFFFFFu);
        ab_move(S, L, L.uid[cu], c % S.W, c / S.W);
    }
}

__device__ __forceinline__ void harvest_behavior(BS& S, const BL& L, int cu) {
    const int r = closest_of(S, L, cu, true), b = closest_of(S, L, cu, false);
    if (r < 0 || b < 0) return;
    const int k = find_aa(S, L, L.uid[cu]);
    if (k >= 0) {
        const int4 a = L.aa[2 * k], bb = L.aa[2 * k + 1];
        if (aa_kind(a) == AA_HARVEST && a.z == L.uid[r] && bb.x == L.uid[b]) return;
    }
    ab_harvest(S, L, L.uid[cu], L.uid[r], L.uid[b], b);
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

__device__ __forceinline__ void build_if_not_already(BS& S, const BL& L, int cu, int type, Rsv& rs) {
    const int k = find_aa(S, L, L.uid[cu]);
    if (k >= 0) {
        const int4 a = L.aa[2 * k];
        if (aa_kind(a) == AA_BUILD && aa_utype(a) == type) return;
    }
    const int pos = find_building_position(S, L, rs, cu % S.W, cu / S.W);
    ab_build(S, L, L.uid[cu], type, pos % S.W, pos / S.W);   // C/Java division: -1 -> (-1, 0)
    if (rs.n == 0) rs.a = pos;
    else rs.b = pos;
    rs.n++;
}

__device__ __forceinline__ int count_units(const BS& S, const BL& L, int type, bool own) {
    return count_where(S, L, [&](int c) {
        const uint32_t o = L.unit[c];
        return u_type(o) == type && (own ? u_owner(o) == S.player : (u_owner(o) >= 0 && u_owner(o) != S.player));
    });
}

// WorkerRush / LightRush / HeavyRush / RangedRush (+ PO*)
__device__ __forceinline__ void rush_get_action(BS& S, const BL& L, int army, bool po) {
    const int p = S.player, res = p ? S.res[1] : S.res[0];
    const int nworkers = count_units(S, L, WORKER, true), nbases = count_units(S, L, BASE, true),
              nbarracks = count_units(S, L, BARRACKS, true);
    for (int k = 0; k < S.n; k++) {   // bases
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        if (u_type(u) != BASE || u_owner(u) != p || L.act[c] != 0) continue;
        const bool tr = army == WORKER ? res >= ut_cost(WORKER) : nworkers < 1 && res >= ut_cost(WORKER);
        if (tr) ab_train(S, L, L.uid[c], WORKER);
    }
    if (army != WORKER) {   // barracks
        const int t = army;
        for (int k = 0; k < S.n; k++) {
            const int c = L.ucell[k];
            const uint32_t u = L.unit[c];
            if (u_type(u) != BARRACKS || u_owner(u) != p || L.act[c] != 0) continue;
            if (res >= ut_cost(t)) ab_train(S, L, L.uid[c], t);
        }
    }
    for (int k = 0; k < S.n; k++) {   // melee units
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        const int t = u_type(u);
        if (!ut_can_attack(t) || ut_can_harvest(t) || u_owner(u) != p || L.act[c] != 0) continue;
        melee_behavior(S, L, c, po);
    }
    // workers, busy ones included (the list is the tail of the unit list walk)
    auto own_worker = [&](int c) {
        const uint32_t u = L.unit[c];
        return ut_can_harvest(u_type(u)) && u_owner(u) == p;
    };
    const int nf = count_where(S, L, own_worker);
    if (nf > 0) {
        Rsv reserved{0, 0, 0};
        int used = 0, head = 0;   // head: workers taken off the free list
        auto worker = [&](int idx) { return nth_where(S, L, idx, own_worker); };   // idx-th own worker, pgs.units order
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
    translate_actions(S, L);
}


// coacAI: CoacAI's published strategy, restated (oracle/mrts_oracle_ai.c
// coac_get_action; its free choices are fixed by league.db's outcomes)
constexpr int COAC_HARVESTERS_PER_BASE = 2, COAC_EXTRA_WORKERS = 2, COAC_BARRACKS_MIN_WORKERS = 2, COAC_DEFENSE_RADIUS = 8;
__device__ __forceinline__ void coac_get_action(BS& S, const BL& L) {
    const int p = S.player, res = p ? S.res[1] : S.res[0];
    const int nworkers = count_units(S, L, WORKER, true), nbases = count_units(S, L, BASE, true),
              nbarracks = count_units(S, L, BARRACKS, true);
    for (int k = 0; k < S.n; k++) {   // bases
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        if (u_type(u) != BASE || u_owner(u) != p || L.act[c] != 0) continue;
        if (nworkers < COAC_HARVESTERS_PER_BASE * nbases + COAC_EXTRA_WORKERS && res >= ut_cost(WORKER)) ab_train(S, L, L.uid[c], WORKER);
    }
    const int t = count_units(S, L, LIGHT, false) > count_units(S, L, RANGED, false) + count_units(S, L, HEAVY, false) ? HEAVY : RANGED;
    for (int k = 0; k < S.n; k++) {   // barracks
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        if (u_type(u) != BARRACKS || u_owner(u) != p || L.act[c] != 0) continue;
        if (res >= ut_cost(t)) ab_train(S, L, L.uid[c], t);
    }
    for (int k = 0; k < S.n; k++) {   // army
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        const int ty = u_type(u);
        if (!ut_can_attack(ty) || ut_can_harvest(ty) || u_owner(u) != p || L.act[c] != 0) continue;
        melee_behavior(S, L, c, false);
    }
    auto own_worker = [&](int c) {
        const uint32_t u = L.unit[c];
        return ut_can_harvest(u_type(u)) && u_owner(u) == p;
    };
    const int nf = count_where(S, L, own_worker);
    if (nf > 0) {
        Rsv reserved{0, 0, 0};
        int used = 0, head = 0;
        auto worker = [&](int idx) { return nth_where(S, L, idx, own_worker); };
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
            const int w = worker(k);
            if (k - head < nh) {
                harvest_behavior(S, L, w);
                continue;
            }
            // defenders: the closest enemy when it is near the worker's closest own base
            const int e = closest_enemy(S, L, w);
            if (e < 0) continue;
            const int b = closest_of(S, L, w, false);
            if (b < 0 || iabs(b % S.W - e % S.W) + iabs(b / S.W - e / S.W) <= COAC_DEFENSE_RADIUS) ab_attack(S, L, L.uid[w], L.uid[e]);
            else harvest_behavior(S, L, w);
        }
    }
    translate_actions(S, L);
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
    for (int i = threadIdx.x; i < posw; i += BT) L.pab[i] = L.pend[i];
    for (int k = 0; k < S.n; k++) {
        const int c = L.ucell[k];
        const uint32_t u = L.unit[c];
        if (u_owner(u) != S.player || L.act[c] != 0) continue;
        int total = 0;
        unit_actions(S, L, c, [&](int, int w) { total += w; });
        uint32_t ctr[4] = {(uint32_t)L.uid[c], S.tick, (uint32_t)S.game, 0x52414E44u + (uint32_t)(1 - S.player)};
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
    }
}


// RandomBiasedSingleUnitAI (randomAI): one unit acts at a time (oracle
// random_single_get_action): nothing while a unit of the player is busy, else
// one idle unit drawn uniformly gets a RandomBiasedAI-weighted action
__device__ __forceinline__ void random_single_get_action(BS& S, const BL& L) {
    auto own = [&](int c) { return u_owner(L.unit[c]) == S.player; };
    if (count_where(S, L, [&](int c) { return own(c) && L.act[c] != 0; }) > 0) return;
    const int ni = count_where(S, L, own);
    if (ni == 0) return;
    S.pa_res[0] = S.pend_res[0];
    S.pa_res[1] = S.pend_res[1];
    const int posw = (S.HW + 2 * S.W) / 32 + 1;
    for (int i = threadIdx.x; i < posw; i += BT) L.pab[i] = L.pend[i];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    uint32_t ctr[4] = {0xFFFFFFFFu, S.tick, (uint32_t)S.game, 0x52534E47u + (uint32_t)(1 - S.player)};
    philox_b(ctr, 0x5EED5EEDu, 0xB0B0B0B0u);
    const int c = nth_where(S, L, (int)(((uint64_t)ctr[1] * (uint32_t)ni) >> 32), own);
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
// ai.getAction(player, gs) of bot game b, by ONE wavefront (lanes = threadIdx.x
// 0..63), LDS at `smem` (bot_lds_bytes).  FUSED: run by wave 0 of a k_step
// workgroup for the NEXT tick while the other waves stream the outputs (no
// workgroup barriers here then; the game state was stored before the caller's
// last barrier); otherwise the body of k_bot (a one-wave workgroup).
template <bool FUSED>
__device__ __forceinline__ void bot_game(const EngineParams& p, int b, int player, unsigned char* smem) {
    const int g = p.nsp_games + b, lane = threadIdx.x;
    const int HW = p.HW, W = p.W;
    int32_t* genv = p.genv + (size_t)g * MRTS_GENV_WORDS;
    const int w_aa = player ? MRTS_G_AA_N : MRTS_G_AA_N0, w_npa = player ? MRTS_G_NPA : MRTS_G_NPA0;
    BS S;
    S.ai = player ? p.bot_ai[b] : (p.bot_ai0 ? p.bot_ai0[b] : -1);
    if (S.ai < 0) return;            // the agent plays this side
    if (S.ai == MRTS_AI_PASSIVE) {   // PassiveAI: all NONE (k_step's fill)
        if (lane0()) genv[w_npa] = 0;
        return;
    }
    BL L = bot_carve(smem, HW, W);
    int4* const aa_g = p.aa + ((size_t)b * 2 + player) * HW * 2;
    int32_t* const pa_g = p.botpa + ((size_t)b * 2 + player) * HW;
    S.W = W;
    S.H = p.H;
    S.HW = HW;
    S.player = player;
    S.partial = p.partial_obs;
    S.game = p.game_offset + g;
    S.tick = (uint32_t)genv[MRTS_G_TICKS];
    S.res[0] = genv[MRTS_G_RES0];
    S.res[1] = genv[MRTS_G_RES1];
    S.naa = genv[w_aa];
    S.npa = 0;
    S.pa_res[0] = S.pa_res[1] = 0;
    const int map = genv[MRTS_G_MAP];
    const int posw = (HW + 2 * W) / 32 + 1, visw = HW / 32 + 1;
    for (int c = lane; c < HW; c += BT) {
        int4 v = p.cells[(size_t)g * HW + c];
        L.unit[c] = (uint32_t)v.x;
        L.uid[c] = v.y;
        L.act[c] = (uint32_t)v.z;
        L.wall[c] = p.map_wall[(size_t)map * HW + c];
    }
    for (int i = lane; i < posw; i += BT) L.pend[i] = L.pab[i] = 0;
    for (int i = lane; i < visw; i += BT) L.vis[i] = 0;
    for (int i = lane; i < 2 * S.naa; i += BT) L.aa[i] = aa_g[i];
    if (lane < 3) L.sc[lane] = 0;   // pending produce cost per player, error bits
    bot_sync<FUSED>();
    // cells observable by the bot's player (PartiallyObservableGameState);
    // read only under partial observability (hidden units, PO* exploration)
    for (int c = lane; S.partial && c < HW; c += BT) {
        const uint32_t u = L.unit[c];
        if (u == 0 || u_owner(u) != S.player) continue;
        const int r = ut_sight(u_type(u)), x = c % W, y = c / W;
        for (int dy = -r; dy <= r; dy++)
            for (int dx = -r; dx <= r; dx++) {
                const int xx = x + dx, yy = y + dy;
                if (xx < 0 || yy < 0 || xx >= W || yy >= p.H || dx * dx + dy * dy > r * r) continue;
                const int cc = yy * W + xx;
                atomicOr(&L.vis[cc >> 5], 1u << (cc & 31));
            }
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
    for (int c = lane; c < HW; c += BT) {
        const uint32_t a = L.act[c];
        if (a == 0) continue;
        const int code = act_code(a), t = code_type(code);
        if (t != A_MOVE && t != A_PRODUCE) continue;
        RU r = usage(S, c, code, u_owner(L.unit[c]));
        atomicOr(&L.pend[(r.pos + W) >> 5], 1u << ((r.pos + W) & 31));
        if (t == A_PRODUCE) atomicAdd(&L.sc[u_owner(L.unit[c])], u_owner(L.unit[c]) ? r.res[1] : r.res[0]);
    }
    // units in pgs.units order: ordered compaction by cell, then rank by uid
    int n = 0;
    for (int base = 0; base < HW; base += BT) {
        const int c = base + lane;
        const bool has = c < HW && L.unit[c] != 0;
        const unsigned long long m = __ballot(has);
        if (has) L.pa[n + __popcll(m & ((1ull << lane) - 1ull))] = c;
        n += __popcll(m);
    }
    bot_sync<FUSED>();
    if (n <= BT) {   // rank by uid with the uids in registers (one per lane)
        const int c = lane < n ? L.pa[lane] : 0, u = lane < n ? L.uid[c] : 0x7fffffff;
        int r = 0;
        for (int j = 0; j < n; j++) r += __shfl(u, j) < u;
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
    S.pend_res[0] = L.sc[0];
    S.pend_res[1] = L.sc[1];
    // lane y: free cells of row y, from one ballot per 64 cells (staged in L.pa,
    // free until the PlayerAction is built)
    S.rurow = 0;
    {
        uint32_t* fw = reinterpret_cast<uint32_t*>(L.pa);
        const int nwords = (HW + 63) / 64 * 2;
        for (int base = 0; base < HW; base += BT) {
            const int c = base + lane;
            const unsigned long long m = __ballot(c < HW && !L.wall[c] && L.unit[c] == 0);
            if (lane == 0) {
                fw[base / 32] = (uint32_t)m;
                fw[base / 32 + 1] = (uint32_t)(m >> 32);
            }
        }
        if (lane == 0) fw[nwords] = 0u;   // the row window's upper word past the last cell
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        S.frow = 0;
        if (lane < p.H) {
            const int o = lane * W, q = o >> 5;
            const uint64_t win = ((uint64_t)fw[q + 1] << 32) | fw[q];
            S.frow = (uint32_t)(win >> (o & 31)) & (W == 32 ? 0xFFFFFFFFu : ((1u << W) - 1u));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    // the closest enemy of every unit (the scan closest_enemy would do, all
    // units at once; the state is fixed during getAction): L.pa[cell], staged
    // like the rows above (-1 = none)
    for (int k = lane; S.ai != MRTS_AI_RANDOM_BIASED && S.ai != MRTS_AI_RANDOM && k < n; k += BT) {
        const int cu = L.ucell[k], me = u_owner(L.unit[cu]), ux = cu % W, uy = cu / W;
        unsigned long long key = ~0ull;
        for (int j = 0; j < n; j++) {
            const int c = L.ucell[j];
            const int o = u_owner(L.unit[c]);
            if (o < 0 || o == me) continue;
            const unsigned d = (unsigned)(iabs(c % W - ux) + iabs(c / W - uy));
            const unsigned long long kk = ((unsigned long long)d << 32) | (unsigned)j;
            key = kk < key ? kk : key;
        }
        L.pa[cu] = key == ~0ull ? -1 : L.ucell[(int)(key & 0xFFFFFFFFu)];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    switch (S.ai) {
    case MRTS_AI_WORKER_RUSH: rush_get_action(S, L, WORKER, false); break;
    case MRTS_AI_LIGHT_RUSH: rush_get_action(S, L, LIGHT, false); break;
    case MRTS_AI_PO_WORKER_RUSH: rush_get_action(S, L, WORKER, true); break;
    case MRTS_AI_PO_LIGHT_RUSH: rush_get_action(S, L, LIGHT, true); break;
    case MRTS_AI_PO_HEAVY_RUSH: rush_get_action(S, L, HEAVY, true); break;
    case MRTS_AI_PO_RANGED_RUSH: rush_get_action(S, L, RANGED, true); break;
    case MRTS_AI_COAC: coac_get_action(S, L); break;
    case MRTS_AI_RANDOM_BIASED: random_biased_get_action(S, L); break;
    case MRTS_AI_RANDOM: random_single_get_action(S, L); break;
    default: break;
    }
    bot_sync<FUSED>();
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
