// mrts_rules.h -- device-side game rules shared by the engine kernels
// (mrts_engine.hip) and the scripted-opponent kernel (mrts_bots.hip):
// rts.units.UnitTypeTable() (VERSION_ORIGINAL), the packed cell / action
// words of mrts_layout.h, Unit.getUnitActions membership (legal_code),
// UnitAction.getValidActionArray (cell_mask) and the one-hot encoder of
// vec_env.py:311-321 (cell_onehot).
#ifndef MRTS_RULES_H
#define MRTS_RULES_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrts_layout.h"

namespace mrts {

// ---------------------------------------------------------------------------
// rts.units.UnitTypeTable() -- VERSION_ORIGINAL (+ UnitType field defaults).
enum { RESOURCE = 0, BASE, BARRACKS, WORKER, LIGHT, HEAVY, RANGED };
enum { A_NONE = 0, A_MOVE, A_HARVEST, A_RETURN, A_PRODUCE, A_ATTACK };

__device__ __forceinline__ int ut_cost(int t) { return t == BASE ? 10 : t == BARRACKS ? 5 : (t >= LIGHT ? 2 : 1); }
__device__ __forceinline__ int ut_hp(int t) { return t == BASE ? 10 : (t == BARRACKS || t == LIGHT || t == HEAVY) ? 4 : 1; }
__device__ __forceinline__ int ut_damage(int t) { return t == LIGHT ? 2 : t == HEAVY ? 4 : 1; }
__device__ __forceinline__ int ut_range(int t) { return t == RANGED ? 3 : 1; }
__device__ __forceinline__ int ut_produce_time(int t) {
    return t == BASE ? 250 : t == BARRACKS ? 200 : t == WORKER ? 50 : t == LIGHT ? 80 : t == HEAVY ? 120 : t == RANGED ? 100 : 10;
}
__device__ __forceinline__ int ut_move_time(int t) { return t == LIGHT ? 8 : t == HEAVY ? 12 : 10; }
__device__ __forceinline__ int ut_attack_time(int t) { return t >= WORKER ? 5 : 10; }
__device__ __forceinline__ int ut_harvest_time(int t) { return t == WORKER ? 20 : 10; }
__device__ __forceinline__ int ut_return_time(int) { return 10; }
__device__ __forceinline__ int ut_harvest_amount(int) { return 1; }
__device__ __forceinline__ int ut_sight(int t) {
    return t == BASE ? 5 : (t == BARRACKS || t == WORKER || t == RANGED) ? 3 : (t == LIGHT || t == HEAVY) ? 2 : 0;
}
// PartiallyObservableGameState: OR the sight disk of a unit at (x, y) (cells with
// dx^2 + dy^2 <= r^2 inside the map) into the bitmap vq (bit c = cell c), one
// span per row: a row's cells are consecutive bits, so each dy costs one
// atomicOr per 32-bit word the span touches (<= 2 for W <= 32) instead of one
// per cell (a base's 81 -> 11).
__device__ __forceinline__ void or_sight_disk(uint32_t* vq, int x, int y, int r, int W, int H) {
    for (int dy = -r; dy <= r; dy++) {
        const int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        int w = r;
        while (w * w + dy * dy > r * r) w--;   // the row's half-width (r <= 5)
        const int b0 = yy * W + max(x - w, 0), b1 = yy * W + min(x + w, W - 1);   // inclusive bit span
        for (int wd = b0 >> 5; wd <= (b1 >> 5); wd++) {
            const int lo = max(b0 - 32 * wd, 0), hi = min(b1 - 32 * wd, 31);
            const uint32_t m = (hi - lo == 31 ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1u)) << lo;
            atomicOr(&vq[wd], m);
        }
    }
}
__device__ __forceinline__ bool ut_can_move(int t) { return t >= WORKER; }
__device__ __forceinline__ bool ut_can_attack(int t) { return t >= WORKER; }
__device__ __forceinline__ bool ut_can_harvest(int t) { return t == WORKER; }
__device__ __forceinline__ bool ut_is_stockpile(int t) { return t == BASE; }
// bitmask of produced unit types
__device__ __forceinline__ int ut_produces(int t) {
    return t == BASE ? (1 << WORKER) : t == BARRACKS ? ((1 << LIGHT) | (1 << HEAVY) | (1 << RANGED)) : t == WORKER ? ((1 << BASE) | (1 << BARRACKS)) : 0;
}

// ---------------------------------------------------------------------------
// Packed words (mrts_layout.h)
__device__ __forceinline__ int u_type(uint32_t w) { return (int)(w & 15u) - 1; }
__device__ __forceinline__ int u_owner(uint32_t w) { return (int)((w >> 4) & 3u) - 1; }
__device__ __forceinline__ int u_hp(uint32_t w) { return (int)((w >> 6) & 1023u); }
__device__ __forceinline__ int u_res(uint32_t w) { return (int)(w >> 16); }
__device__ __forceinline__ uint32_t u_make(int type, int owner, int hp, int res) {
    return (uint32_t)(type + 1) | ((uint32_t)(owner + 1) << 4) | ((uint32_t)hp << 6) | ((uint32_t)res << 16);
}
__device__ __forceinline__ uint32_t u_with_hp(uint32_t w, int hp) { return (w & ~(1023u << 6)) | ((uint32_t)hp << 6); }
__device__ __forceinline__ uint32_t u_with_res(uint32_t w, int res) { return (w & 0xFFFFu) | ((uint32_t)res << 16); }

// action code (12 bits): type | param << 3 | utype << 9 ; action word = code + 1 | (done + 1) << 12
__device__ __forceinline__ int code_make(int type, int param, int utype) { return type | (param << 3) | (utype << 9); }
__device__ __forceinline__ int code_type(int code) { return code & 7; }
__device__ __forceinline__ int code_param(int code) { return (code >> 3) & 63; }
__device__ __forceinline__ int code_utype(int code) { return (code >> 9) & 7; }
__device__ __forceinline__ uint32_t act_make(int code, int done) { return (uint32_t)(code + 1) | ((uint32_t)(done + 1) << 12); }
__device__ __forceinline__ int act_code(uint32_t a) { return (int)(a & 0xFFFu) - 1; }
__device__ __forceinline__ int act_done(uint32_t a) { return (int)(a >> 12) - 1; }
__device__ __forceinline__ uint32_t seq_make(int time, int player, int rank) {
    return ((uint32_t)time << 13) | ((uint32_t)player << 12) | (uint32_t)rank;
}
__device__ __forceinline__ int seq_time(uint32_t s) { return (int)(s >> 13); }

// UnitAction.ETA for a non-NONE code executed by a unit of type t
__device__ __forceinline__ int eta_code(int code, int t) {
    switch (code_type(code)) {
    case A_MOVE: return ut_move_time(t);
    case A_HARVEST: return ut_harvest_time(t);
    case A_RETURN: return ut_return_time(t);
    case A_PRODUCE: return ut_produce_time(code_utype(code));
    case A_ATTACK: return ut_attack_time(t);
    }
    return 0;
}

__device__ __forceinline__ int dir_dx(int d) { return d == 1 ? 1 : d == 3 ? -1 : 0; }
__device__ __forceinline__ int dir_dy(int d) { return d == 2 ? 1 : d == 0 ? -1 : 0; }

struct Grid {
    int W, H, HW;
};

// neighbour cell in direction d, or -1 when off the map
__device__ __forceinline__ int nb_cell(const Grid& gd, int c, int d) {
    int x = c % gd.W + dir_dx(d), y = c / gd.W + dir_dy(d);
    return (x < 0 || y < 0 || x >= gd.W || y >= gd.H) ? -1 : y * gd.W + x;
}

// Unit.getUnitActions membership test (UnitAction.equals), i.e.
// Unit.canExecuteAction for a decoded action code of the unit at cell c.
__device__ inline bool legal_code(const Grid& gd, int c, int code, const uint32_t* s_unit, const uint8_t* s_wall, int res_player) {
    uint32_t u = s_unit[c];
    int t = u_type(u), owner = u_owner(u);
    int type = code_type(code), param = code_param(code);
    switch (type) {
    case A_NONE: return true;
    case A_MOVE: {
        if (!ut_can_move(t)) return false;
        int n = nb_cell(gd, c, param);
        return n >= 0 && !s_wall[n] && s_unit[n] == 0;
    }
    case A_HARVEST: {
        if (!ut_can_harvest(t) || u_res(u) != 0) return false;
        int n = nb_cell(gd, c, param);
        return n >= 0 && s_unit[n] != 0 && u_type(s_unit[n]) == RESOURCE;
    }
    case A_RETURN: {
        if (!ut_can_harvest(t) || u_res(u) <= 0) return false;
        int n = nb_cell(gd, c, param);
        return n >= 0 && s_unit[n] != 0 && ut_is_stockpile(u_type(s_unit[n])) && u_owner(s_unit[n]) == owner;
    }
    case A_PRODUCE: {
        int ut = code_utype(code);
        if (!((ut_produces(t) >> ut) & 1) || res_player < ut_cost(ut)) return false;
        int n = nb_cell(gd, c, param);
        return n >= 0 && !s_wall[n] && s_unit[n] == 0;
    }
    case A_ATTACK: {
        if (!ut_can_attack(t)) return false;
        int dx = param % MRTS_ATTACK_GRID - MRTS_ATTACK_GRID / 2, dy = param / MRTS_ATTACK_GRID - MRTS_ATTACK_GRID / 2;
        int r = ut_range(t);
        if (dx * dx + dy * dy > r * r) return false;
        int x = c % gd.W + dx, y = c / gd.W + dy;
        if (x < 0 || y < 0 || x >= gd.W || y >= gd.H) return false;
        uint32_t o = s_unit[y * gd.W + x];
        int oo = u_owner(o);
        return o != 0 && oo >= 0 && oo != owner;
    }
    }
    return false;
}

// UnitAction.getValidActionArray for the idle unit at c: 79 bits (bit 0 = source)
__device__ inline void cell_mask(const Grid& gd, int c, int player, const uint32_t* s_unit, const uint32_t* s_act,
                          const uint8_t* s_wall, int res_player, uint32_t m[3]) {
    m[0] = m[1] = m[2] = 0;
    uint32_t u = s_unit[c];
    if (u == 0 || u_owner(u) != player || s_act[c] != 0) return;
    auto setb = [&](int b) { m[b >> 5] |= 1u << (b & 31); };
    const int T = 1, MV = 7, HV = 11, RT = 15, PD = 19, PT = 23, AT = 30;
    setb(0);
    setb(T + A_NONE);
    int t = u_type(u), x = c % gd.W, y = c / gd.W;
    int nb[4];
    bool freec[4];
    for (int d = 0; d < 4; d++) {
        nb[d] = nb_cell(gd, c, d);
        freec[d] = nb[d] >= 0 && !s_wall[nb[d]] && s_unit[nb[d]] == 0;
    }
    const int cc = MRTS_ATTACK_GRID / 2;
    if (ut_can_attack(t)) {
        int r = ut_range(t);
        for (int dy = -r; dy <= r; dy++)
            for (int dx = -r; dx <= r; dx++) {
                if (dx * dx + dy * dy > r * r) continue;
                int xx = x + dx, yy = y + dy;
                if (xx < 0 || yy < 0 || xx >= gd.W || yy >= gd.H) continue;
                uint32_t o = s_unit[yy * gd.W + xx];
                int oo = u_owner(o);
                if (o != 0 && oo >= 0 && oo != player) {
                    setb(T + A_ATTACK);
                    setb(AT + (cc + dy) * MRTS_ATTACK_GRID + (cc + dx));
                }
            }
    }
    if (ut_can_harvest(t)) {
        int ur = u_res(u);
        for (int d = 0; d < 4; d++) {
            if (nb[d] < 0 || s_unit[nb[d]] == 0) continue;
            uint32_t o = s_unit[nb[d]];
            if (ur == 0 && u_type(o) == RESOURCE) {
                setb(T + A_HARVEST);
                setb(HV + d);
            }
            if (ur > 0 && ut_is_stockpile(u_type(o)) && u_owner(o) == player) {
                setb(T + A_RETURN);
                setb(RT + d);
            }
        }
    }
    int prod = ut_produces(t);
    bool anyfree = freec[0] || freec[1] || freec[2] || freec[3];
    if (prod && anyfree) {
        for (int ut = 0; ut < MRTS_NTYPES; ut++) {
            if (!((prod >> ut) & 1) || res_player < ut_cost(ut)) continue;
            setb(T + A_PRODUCE);
            setb(PT + ut);
            for (int d = 0; d < 4; d++)
                if (freec[d]) setb(PD + d);
        }
    }
    if (ut_can_move(t) && anyfree) {
        setb(T + A_MOVE);
        for (int d = 0; d < 4; d++)
            if (freec[d]) setb(MV + d);
    }
}

// one-hot word of vec_env.py:311-321 for the cell (perspective `player`).
// Partial observability (P == 31, PartiallyObservableGameState): `shown` is 0
// for a unit the player cannot see (the cell reads as empty); bits 29/30 are
// the visibility plane: the shown unit is visible to the opponent.
__device__ __forceinline__ uint32_t cell_onehot(uint32_t u, uint32_t a, uint8_t wall, int player, int P = 29,
                                                bool shown = true, bool opp_sees = false) {
    uint32_t b = 0;
    if (!shown) u = 0;
    if (P == 31) b |= 1u << (29 + ((u != 0 && opp_sees) ? 1 : 0));
    if (u == 0) {
        b |= 1u | (1u << 5) | (1u << 10) | (1u << 13) | (1u << 21);
    } else {
        int hp = min(max(u_hp(u), 0), 4), res = min(u_res(u), 4), ow = u_owner(u);
        int rel = ow < 0 ? 0 : (ow == player ? 1 : 2);
        int at = a ? min(code_type(act_code(a)), 5) : 0;
        b |= (1u << hp) | (1u << (5 + res)) | (1u << (10 + rel)) | (1u << (13 + u_type(u) + 1)) | (1u << (21 + at));
    }
    return b | (1u << (27 + (wall ? 1 : 0)));
}

}  // namespace mrts
#endif
