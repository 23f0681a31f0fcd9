/*
 * mrts_oracle.c -- CPU restatement of the MicroRTS engine and of the gym-microrts
 * JNI vector client.  TEST INFRASTRUCTURE ONLY (see mrts_oracle.h).
 *
 * Every Java class named below lives in the absent git submodule
 * gym_microrts/microrts (adFrej/MicroRTS-KG @ unknown commit, santiontanon/microrts
 * lineage; /root/reference/.gitmodules:1-3).  Its behaviour is restated from the
 * public engine; the reference's own call sites are cited as file:line into
 * /root/reference.  Rules pinned by the reference tests are marked PINNED, the
 * rest follow SURVEY.md Appendix A and DESIGN.md §4 (UNPINNED).
 */
#include "mrts_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* rts.units.UnitTypeTable() = VERSION_ORIGINAL, MOVE_CONFLICT_RESOLUTION_CANCEL_BOTH
 * (constructed at vec_env.py:172-174).  UnitType field defaults (cost 1, hp 1,
 * damage 1, range 1, all times 10, harvestAmount 1, sight 4) apply where the
 * table does not set a value.                                                */
enum { T_RESOURCE = 0, T_BASE, T_BARRACKS, T_WORKER, T_LIGHT, T_HEAVY, T_RANGED, NTYPES };
typedef struct {
    int cost, hp, min_dmg, max_dmg, range, produce_t, move_t, attack_t, harvest_t, return_t,
        harvest_amt, sight;
    int is_resource, is_stockpile, can_harvest, can_move, can_attack;
    int nprod, prod[3];
} OType;
static const OType UT[NTYPES] = {
    /* Resource */ {1, 1, 1, 1, 1, 10, 10, 10, 10, 10, 1, 0, 1, 0, 0, 0, 0, 0, {0}},
    /* Base     */ {10, 10, 1, 1, 1, 250, 10, 10, 10, 10, 1, 5, 0, 1, 0, 0, 0, 1, {T_WORKER}},
    /* Barracks */ {5, 4, 1, 1, 1, 200, 10, 10, 10, 10, 1, 3, 0, 0, 0, 0, 0, 3, {T_LIGHT, T_HEAVY, T_RANGED}},
    /* Worker   */ {1, 1, 1, 1, 1, 50, 10, 5, 20, 10, 1, 3, 0, 0, 1, 1, 1, 2, {T_BASE, T_BARRACKS}},
    /* Light    */ {2, 4, 2, 2, 1, 80, 8, 5, 10, 10, 1, 2, 0, 0, 0, 1, 1, 0, {0}},
    /* Heavy    */ {2, 4, 4, 4, 1, 120, 12, 5, 10, 10, 1, 2, 0, 0, 0, 1, 1, 0, {0}},
    /* Ranged   */ {2, 1, 1, 1, 3, 100, 10, 5, 10, 10, 1, 3, 0, 0, 0, 1, 1, 0, {0}},
};
#define MAX_HW_ORACLE 4096
#define MAX_ATTACK_RANGE 3 /* UnitTypeTable.getMaxAttackRange(); 7x7 grid at vec_env.py:234 */
#define ATTACK_GRID 7

/* rts.UnitAction */
enum { A_NONE = 0, A_MOVE, A_HARVEST, A_RETURN, A_PRODUCE, A_ATTACK };
enum { D_UP = 0, D_RIGHT, D_DOWN, D_LEFT };
#define DIRECTION_NONE (-1)
typedef struct {
    int type;
    int param; /* direction, or the duration of a NONE action                */
    int x, y;  /* attack location                                            */
    int utype; /* produced unit type                                         */
} OAct;

/* rts.units.Unit (slot pool in insertion order = PhysicalGameState.units) */
typedef struct {
    int alive;
    int type, player, x, y, hp, res;
    int assign; /* slot in the assignment list, -1 if none                   */
} OUnit;

/* rts.UnitActionAssignment inside GameState.unitActions (a LinkedHashMap). */
typedef struct {
    int alive;
    int unit;
    OAct act;
    int time;
} OAssign;

/* rts.ResourceUsage: positionsUsed list + resourcesUsed[2] */
typedef struct {
    int npos, cap;
    int *pos;
    int res[2];
    int inl[2]; /* inline storage for single-action usages                 */
} ORU;

typedef struct {
    int unit;
    OAct act;
} OPair;
typedef struct { /* rts.PlayerAction */
    OPair *e;
    int n, cap;
    ORU ru;
} OPA;

typedef struct { /* rts.GameState + rts.PhysicalGameState */
    int W, H;
    const uint8_t *terrain;
    int res[2];
    int time;
    OUnit *u;
    int nu, capu;
    int *grid; /* cell -> unit slot, -1 if empty                              */
    OAssign *as;
    int na, capa;
    int64_t ev[OEV_N]; /* event counters (ovec_event_counts); survive resets       */
} OGS;

struct OVec {
    int nsp, nbot, ngames, nenvs, max_steps, partial_obs;
    int W, H;
    OMap *maps;
    int nmaps;
    int *game_map;
    int *bot_ai;
    int *bot_ai0;   /* per bot env: ai1 of a bot-vs-bot game, -1 = the agent plays p0 */
    OGS *gs;
    int *env_steps; /* per game (selfplay pairs step together)                */
    uint32_t *ticks;/* per game: steps since creation (bot RNG counter)        */
    struct OAAMapS *aam; /* per game: the bot's AbstractionLayerAI.actions     */
    int32_t *raw;   /* [N][P_raw][H][W] last response observation             */
};

/* ------------------------------------------------------------------------- */
static void *xrealloc(void *p, size_t n) {
    void *q = realloc(p, n);
    if (!q && n) {
        fprintf(stderr, "oracle: out of memory\n");
        abort();
    }
    return q;
}

static int eta(const OUnit *u, const OAct *a) { /* UnitAction.ETA */
    switch (a->type) {
    case A_NONE: return a->param;
    case A_MOVE: return UT[u->type].move_t;
    case A_ATTACK: return UT[u->type].attack_t;
    case A_HARVEST: return UT[u->type].harvest_t;
    case A_RETURN: return UT[u->type].return_t;
    case A_PRODUCE: return UT[a->utype].produce_t;
    }
    return 0;
}

static OAct act_none(int duration) {
    OAct a = {A_NONE, duration, 0, 0, -1};
    return a;
}

static int act_eq(const OAct *a, const OAct *b) { /* UnitAction.equals */
    if (a->type != b->type) return 0;
    switch (a->type) {
    case A_NONE:
    case A_MOVE:
    case A_HARVEST:
    case A_RETURN: return a->param == b->param;
    case A_ATTACK: return a->x == b->x && a->y == b->y;
    default: return a->param == b->param && a->utype == b->utype;
    }
}

static int terrain_at(const OGS *g, int x, int y) { return g->terrain[y * g->W + x]; }
static int unit_at(const OGS *g, int x, int y) { /* PhysicalGameState.getUnitAt */
    if (x < 0 || y < 0 || x >= g->W || y >= g->H) return -1;
    return g->grid[y * g->W + x];
}

/* ---- ResourceUsage ------------------------------------------------------ */
static void ru_init(ORU *r) {
    r->npos = 0;
    r->cap = 2;
    r->pos = r->inl;
    r->res[0] = r->res[1] = 0;
}
static void ru_free(ORU *r) {
    if (r->pos != r->inl) free(r->pos);
    ru_init(r);
}
static void ru_add_pos(ORU *r, int p) {
    if (r->npos == r->cap) {
        int nc = r->cap * 2;
        int *np = (int *)malloc(sizeof(int) * nc);
        memcpy(np, r->pos, sizeof(int) * r->npos);
        if (r->pos != r->inl) free(r->pos);
        r->pos = np;
        r->cap = nc;
    }
    r->pos[r->npos++] = p;
}
static int dir_offset(const OGS *g, int dir) {
    switch (dir) {
    case D_UP: return -g->W;
    case D_RIGHT: return 1;
    case D_DOWN: return g->W;
    case D_LEFT: return -1;
    }
    return 0;
}
/* UnitAction.resourceUsage: positions are x + y*W + offset, unchecked. */
static void resource_usage(const OGS *g, const OUnit *u, const OAct *a, ORU *r) {
    ru_init(r);
    if (a->type == A_MOVE) {
        ru_add_pos(r, u->x + u->y * g->W + dir_offset(g, a->param));
    } else if (a->type == A_PRODUCE) {
        r->res[u->player] += UT[a->utype].cost;
        ru_add_pos(r, u->x + u->y * g->W + dir_offset(g, a->param));
    }
}
/* ResourceUsage.consistentWith(another, gs) -- note the pairwise resource test */
static int consistent_with(const ORU *self, const ORU *another, const OGS *g) {
    for (int i = 0; i < another->npos; i++)
        for (int j = 0; j < self->npos; j++)
            if (self->pos[j] == another->pos[i]) return 0;
    for (int i = 0; i < 2; i++) {
        int s = self->res[i] + another->res[i];
        if (s > 0 && s > g->res[i]) return 0;
    }
    return 1;
}
static void ru_merge(ORU *dst, const ORU *src) {
    for (int i = 0; i < src->npos; i++) ru_add_pos(dst, src->pos[i]);
    dst->res[0] += src->res[0];
    dst->res[1] += src->res[1];
}

/* ---- GameState bookkeeping ---------------------------------------------- */
static int add_unit(OGS *g, int type, int player, int x, int y, int res, int hp) {
    if (g->grid[y * g->W + x] >= 0) { /* PhysicalGameState.addUnit throws */
        fprintf(stderr, "oracle: two units in position (%d,%d)\n", x, y);
        abort();
    }
    if (g->nu == g->capu) {
        g->capu = g->capu ? g->capu * 2 : 64;
        g->u = (OUnit *)xrealloc(g->u, sizeof(OUnit) * g->capu);
    }
    OUnit *u = &g->u[g->nu];
    u->alive = 1;
    u->type = type;
    u->player = player;
    u->x = x;
    u->y = y;
    u->res = res;
    u->hp = hp;
    u->assign = -1;
    g->grid[y * g->W + x] = g->nu;
    return g->nu++;
}

static void remove_assign(OGS *g, int ui) { /* unitActions.remove(u) */
    int a = g->u[ui].assign;
    if (a >= 0) {
        g->as[a].alive = 0;
        g->u[ui].assign = -1;
    }
}

static void remove_unit(OGS *g, int ui) { /* GameState.removeUnit */
    OUnit *u = &g->u[ui];
    if (!u->alive) return;
    u->alive = 0;
    g->grid[u->y * g->W + u->x] = -1;
    remove_assign(g, ui);
}

static void put_assign(OGS *g, int ui, const OAct *a, int time) { /* unitActions.put */
    if (g->na == g->capa) {
        /* compact dead entries first (order preserved) */
        int w = 0;
        for (int i = 0; i < g->na; i++) {
            if (!g->as[i].alive) continue;
            g->as[w] = g->as[i];
            g->u[g->as[w].unit].assign = w;
            w++;
        }
        g->na = w;
        if (g->na * 2 >= g->capa) {
            g->capa = g->capa ? g->capa * 2 : 64;
            g->as = (OAssign *)xrealloc(g->as, sizeof(OAssign) * g->capa);
        }
    }
    OAssign *s = &g->as[g->na];
    s->alive = 1;
    s->unit = ui;
    s->act = *a;
    s->time = time;
    g->u[ui].assign = g->na++;
}

static void gs_load(OGS *g, const OMap *m) { /* PhysicalGameState.load + new GameState */
    g->W = m->width;
    g->H = m->height;
    g->terrain = m->terrain;
    g->res[0] = m->player_res[0];
    g->res[1] = m->player_res[1];
    g->time = 0;
    g->nu = 0;
    g->na = 0;
    g->grid = (int *)xrealloc(g->grid, sizeof(int) * g->W * g->H);
    for (int i = 0; i < g->W * g->H; i++) g->grid[i] = -1;
    for (int i = 0; i < m->num_units; i++) {
        const int32_t *r = m->units + 6 * i;
        add_unit(g, r[0], r[1], r[2], r[3], r[4], r[5]);
    }
}

/* ---- Unit.getUnitActions(gs, noneDuration) ------------------------------ */
#define MAXLIST 64
/* getUnitAt in a game state some of whose units are hidden (a bot's
 * PartiallyObservableGameState); hidden == NULL is the full state. */
static int unit_at_h(const OGS *g, const uint8_t *hidden, int x, int y) {
    int i = unit_at(g, x, y);
    return (i >= 0 && hidden && hidden[i]) ? -1 : i;
}
static int unit_actions_h(const OGS *g, const uint8_t *hidden, int ui, int none_duration, OAct *l) {
    const OUnit *u = &g->u[ui];
    const OType *t = &UT[u->type];
    int n = 0, x = u->x, y = u->y;
    int uup = unit_at_h(g, hidden, x, y - 1), uright = unit_at_h(g, hidden, x + 1, y),
        udown = unit_at_h(g, hidden, x, y + 1), uleft = unit_at_h(g, hidden, x - 1, y);
    if (t->can_attack) {
        if (t->range == 1) {
            int nb[4] = {uup, uright, udown, uleft};
            for (int d = 0; d < 4; d++) {
                int o = nb[d];
                if (o >= 0 && g->u[o].player != u->player && g->u[o].player >= 0) {
                    OAct a = {A_ATTACK, DIRECTION_NONE, g->u[o].x, g->u[o].y, -1};
                    l[n++] = a;
                }
            }
        } else {
            int sq = t->range * t->range;
            for (int i = 0; i < g->nu; i++) {
                const OUnit *o = &g->u[i];
                if (!o->alive || (hidden && hidden[i]) || o->player < 0 || o->player == u->player) continue;
                int dx = o->x - x, dy = o->y - y;
                if (dx * dx + dy * dy <= sq) {
                    OAct a = {A_ATTACK, DIRECTION_NONE, o->x, o->y, -1};
                    if (n < MAXLIST) l[n++] = a;
                }
            }
        }
    }
    if (t->can_harvest) {
        int nb[4] = {uup, uright, udown, uleft};
        if (u->res == 0) {
            for (int d = 0; d < 4; d++)
                if (nb[d] >= 0 && UT[g->u[nb[d]].type].is_resource) {
                    OAct a = {A_HARVEST, d, 0, 0, -1};
                    l[n++] = a;
                }
        }
        if (u->res > 0) {
            for (int d = 0; d < 4; d++)
                if (nb[d] >= 0 && UT[g->u[nb[d]].type].is_stockpile && g->u[nb[d]].player == u->player) {
                    OAct a = {A_RETURN, d, 0, 0, -1};
                    l[n++] = a;
                }
        }
    }
    int tup = y > 0 ? terrain_at(g, x, y - 1) : 1;
    int tright = x < g->W - 1 ? terrain_at(g, x + 1, y) : 1;
    int tdown = y < g->H - 1 ? terrain_at(g, x, y + 1) : 1;
    int tleft = x > 0 ? terrain_at(g, x - 1, y) : 1;
    int tt[4] = {tup, tright, tdown, tleft};
    int nb[4] = {uup, uright, udown, uleft};
    for (int k = 0; k < t->nprod; k++) {
        int ut = t->prod[k];
        if (g->res[u->player] >= UT[ut].cost) {
            for (int d = 0; d < 4; d++)
                if (tt[d] == 0 && nb[d] < 0) {
                    OAct a = {A_PRODUCE, d, 0, 0, ut};
                    l[n++] = a;
                }
        }
    }
    if (t->can_move) {
        for (int d = 0; d < 4; d++)
            if (tt[d] == 0 && nb[d] < 0) {
                OAct a = {A_MOVE, d, 0, 0, -1};
                l[n++] = a;
            }
    }
    l[n++] = act_none(none_duration);
    return n;
}
static int unit_actions(const OGS *g, int ui, int none_duration, OAct *l) {
    return unit_actions_h(g, NULL, ui, none_duration, l);
}

static int can_execute(const OGS *g, int ui, const OAct *a) { /* Unit.canExecuteAction */
    OAct l[MAXLIST + 16];
    int n = unit_actions(g, ui, eta(&g->u[ui], a), l);
    for (int i = 0; i < n; i++)
        if (act_eq(&l[i], a)) return 1;
    return 0;
}

/* ---- PlayerAction ------------------------------------------------------- */
static void pa_init(OPA *p) {
    p->e = NULL;
    p->n = p->cap = 0;
    ru_init(&p->ru);
}
static void pa_free(OPA *p) {
    free(p->e);
    ru_free(&p->ru);
    pa_init(p);
}
static void pa_add(OPA *p, int ui, const OAct *a) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 32;
        p->e = (OPair *)xrealloc(p->e, sizeof(OPair) * p->cap);
    }
    p->e[p->n].unit = ui;
    p->e[p->n].act = *a;
    p->n++;
}

/* UnitAction.fromVectorAction.  Returns 0 for a row whose selected component
 * is out of range (the Java raises; see DESIGN.md §4 "invalid rows").       */
static int decode_row(const OGS *g, const OUnit *u, const int64_t *r, OAct *a) {
    int64_t ty = r[0];
    switch (ty) {
    case A_NONE: *a = act_none(1); return 1; /* PINNED jointly with harvest 20 (test_reward.py:36-48) */
    case A_MOVE:
        if (r[1] < 0 || r[1] > 3) return 0;
        a->type = A_MOVE; a->param = (int)r[1]; a->x = a->y = 0; a->utype = -1;
        return 1;
    case A_HARVEST:
        if (r[2] < 0 || r[2] > 3) return 0;
        a->type = A_HARVEST; a->param = (int)r[2]; a->x = a->y = 0; a->utype = -1;
        return 1;
    case A_RETURN:
        if (r[3] < 0 || r[3] > 3) return 0;
        a->type = A_RETURN; a->param = (int)r[3]; a->x = a->y = 0; a->utype = -1;
        return 1;
    case A_PRODUCE:
        if (r[4] < 0 || r[4] > 3 || r[5] < 0 || r[5] >= NTYPES) return 0;
        a->type = A_PRODUCE; a->param = (int)r[4]; a->x = a->y = 0; a->utype = (int)r[5];
        return 1;
    case A_ATTACK: {
        if (r[6] < 0 || r[6] >= ATTACK_GRID * ATTACK_GRID) return 0;
        int c = ATTACK_GRID / 2;
        a->type = A_ATTACK; a->param = DIRECTION_NONE; a->utype = -1;
        a->x = u->x + (int)(r[6] % ATTACK_GRID) - c;
        a->y = u->y + (int)(r[6] / ATTACK_GRID) - c;
        return 1;
    }
    }
    (void)g;
    return 0;
}

/* JNIAI.getAction -> PlayerAction.fromVectorAction + fillWithNones(gs, p, 1).
 * Rows: the python-side rows for cells with source_unit_mask == 1, ascending
 * cell index (vec_env.py:972-974, PINNED order).                            */
static void jni_get_action(OGS *g, int player, const int64_t *act, const int32_t *src, OPA *pa) {
    pa_init(pa);
    int HW = g->W * g->H;
    for (int c = 0; c < HW; c++) {
        if (!src[c]) continue;
        int ui = g->grid[c];
        if (ui < 0) continue;
        OUnit *u = &g->u[ui];
        if (u->player != player || u->assign >= 0) continue;
        OAct a;
        if (!decode_row(g, u, act + 7 * (size_t)c, &a)) continue;
        ORU r;
        resource_usage(g, u, &a, &r);
        if (consistent_with(&r, &pa->ru, g)) {
            ru_merge(&pa->ru, &r);
            pa_add(pa, ui, &a);
        }
        ru_free(&r);
    }
    /* PlayerAction.fillWithNones(gs, player, 1), pgs.units order */
    for (int i = 0; i < g->nu; i++) {
        OUnit *u = &g->u[i];
        if (!u->alive || u->player != player || u->assign >= 0) continue;
        int found = 0;
        for (int k = 0; k < pa->n; k++)
            if (pa->e[k].unit == i) { found = 1; break; }
        if (!found) {
            OAct a = act_none(1);
            pa_add(pa, i, &a);
        }
    }
}

/* ai.PassiveAI.getAction */
static void passive_get_action(OGS *g, int player, OPA *pa) {
    pa_init(pa);
    for (int i = 0; i < g->nu; i++) {
        OUnit *u = &g->u[i];
        if (!u->alive || u->player != player || u->assign >= 0) continue;
        OAct a = act_none(1);
        pa_add(pa, i, &a);
    }
}

/* GameState.issue(pa) */
static void issue(OGS *g, OPA *pa) {
    for (int k = 0; k < pa->n; k++) {
        OPair local = pa->e[k];
        int original = 1; /* is `p` still the Pair object held by pa?     */
        OPair *p = &pa->e[k];
        ORU ru;
        resource_usage(g, &g->u[p->unit], &p->act, &ru);
        for (int i = 0; i < g->na; i++) {
            OAssign *uaa = &g->as[i];
            if (!uaa->alive) continue;
            ORU ur;
            resource_usage(g, &g->u[uaa->unit], &uaa->act, &ur);
            int ok = consistent_with(&ur, &ru, g);
            ru_free(&ur);
            if (ok) continue;
            if (uaa->time == g->time) { /* same cycle: CANCEL_BOTH */
                g->ev[OEV_CANCEL_BOTH]++;
                int d1 = eta(&g->u[uaa->unit], &uaa->act);
                int d2 = eta(&g->u[p->unit], &p->act);
                int d = d1 < d2 ? d1 : d2;
                uaa->act = act_none(d);
                if (original) {
                    local = *p;
                    p = &local;
                    original = 0;
                }
                p->act = act_none(d); /* p = new Pair(...): pa keeps the old action */
            } else {
                /* "Inconsistent actions were executed!": p.m_b = new UnitAction(NONE) */
                g->ev[OEV_INCONSISTENT]++;
                p->act = act_none(DIRECTION_NONE);
            }
        }
        ru_free(&ru);
        put_assign(g, p->unit, &p->act, g->time);
    }
}

/* GameState.issueSafe(pa): illegal -> NONE with the same ETA (in place). */
static void issue_safe(OGS *g, OPA *pa) {
    for (int k = 0; k < pa->n; k++) {
        OPair *p = &pa->e[k];
        if (!can_execute(g, p->unit, &p->act)) p->act = act_none(eta(&g->u[p->unit], &p->act));
    }
    issue(g, pa);
}

/* UnitAction.execute */
static void execute(OGS *g, int ui, const OAct *a) {
    OUnit *u = &g->u[ui];
    switch (a->type) {
    case A_NONE: break;
    case A_MOVE: {
        int nx = u->x, ny = u->y;
        if (a->param == D_UP) ny--;
        else if (a->param == D_RIGHT) nx++;
        else if (a->param == D_DOWN) ny++;
        else if (a->param == D_LEFT) nx--;
        if (u->alive) {
            g->grid[u->y * g->W + u->x] = -1;
            if (g->grid[ny * g->W + nx] >= 0) {
                fprintf(stderr, "oracle: move into occupied cell\n");
                abort();
            }
            g->grid[ny * g->W + nx] = ui;
        }
        u->x = nx;
        u->y = ny;
        break;
    }
    case A_ATTACK: {
        int o = unit_at(g, a->x, a->y);
        if (o >= 0) {
            /* VERSION_ORIGINAL: minDamage == maxDamage, no RNG draw */
            g->u[o].hp -= UT[u->type].min_dmg;
            if (u->player >= 0) g->ev[OEV_HITS + u->player]++;
            if (g->u[o].hp <= 0) {
                if (u->player >= 0) g->ev[OEV_KILLS + u->player]++;
                remove_unit(g, o);
            }
        }
        break;
    }
    case A_HARVEST: {
        int tx = u->x + (a->param == D_RIGHT) - (a->param == D_LEFT);
        int ty = u->y + (a->param == D_DOWN) - (a->param == D_UP);
        int r = unit_at(g, tx, ty);
        if (r >= 0 && UT[g->u[r].type].is_resource && UT[u->type].can_harvest && u->res == 0) {
            g->u[r].res -= UT[u->type].harvest_amt;
            if (g->u[r].res <= 0) remove_unit(g, r);
            u->res = UT[u->type].harvest_amt;
        }
        break;
    }
    case A_RETURN: {
        int tx = u->x + (a->param == D_RIGHT) - (a->param == D_LEFT);
        int ty = u->y + (a->param == D_DOWN) - (a->param == D_UP);
        int b = unit_at(g, tx, ty);
        if (b >= 0 && UT[g->u[b].type].is_stockpile && u->res > 0) {
            g->res[u->player] += u->res;
            u->res = 0;
        }
        break;
    }
    case A_PRODUCE: {
        int tx = u->x + (a->param == D_RIGHT) - (a->param == D_LEFT);
        int ty = u->y + (a->param == D_DOWN) - (a->param == D_UP);
        int owner = u->player; /* add_unit may move the unit pool */
        if (owner >= 0) g->ev[OEV_PRODUCED + 7 * owner + a->utype]++;
        add_unit(g, a->utype, owner, tx, ty, 0, UT[a->utype].hp);
        g->res[owner] -= UT[a->utype].cost;
        break;
    }
    }
}

/* PhysicalGameState.gameover / winner */
static int gs_winner(const OGS *g, int *gameover) {
    int cnt[2] = {0, 0};
    for (int i = 0; i < g->nu; i++)
        if (g->u[i].alive && g->u[i].player >= 0) cnt[g->u[i].player]++;
    int winner = -1, multi = 0;
    for (int p = 0; p < 2; p++)
        if (cnt[p] > 0) {
            if (winner == -1) winner = p;
            else multi = 1;
        }
    if (multi) winner = -1;
    *gameover = (cnt[0] + cnt[1] == 0) || (!multi && winner != -1);
    return winner;
}

/* GameState.cycle() */
static int cycle(OGS *g) {
    g->time++;
    int nready = 0;
    int *ready = (int *)malloc(sizeof(int) * (g->na + 1));
    for (int i = 0; i < g->na; i++) {
        OAssign *s = &g->as[i];
        if (s->alive && eta(&g->u[s->unit], &s->act) + s->time <= g->time) ready[nready++] = i;
    }
    /* copy out first: executing may compact nothing (no puts during cycle) */
    for (int k = 0; k < nready; k++) {
        OAssign s = g->as[ready[k]];
        remove_assign(g, s.unit);
        execute(g, s.unit, &s.act);
    }
    free(ready);
    int go;
    gs_winner(g, &go);
    return go;
}

/* ai.reward.* computeReward(maxplayer, minplayer, te, afterGs): channels
 * WinLoss, ResourceGather, ProduceWorker, ProduceBuilding, Attack,
 * ProduceCombatUnit (vec_env.py:185-195).  te holds the issued PlayerActions
 * as left by issueSafe.                                                      */
static void rewards(const OGS *g, const OPA *pa0, const OPA *pa1, int maxplayer, int gameover,
                    int winner, double *r, uint8_t *d) {
    for (int i = 0; i < 6; i++) r[i] = 0.0;
    const OPA *pas[2] = {pa0, pa1};
    for (int q = 0; q < 2; q++) {
        const OPA *pa = pas[q];
        for (int k = 0; k < pa->n; k++) {
            const OUnit *u = &g->u[pa->e[k].unit];
            const OAct *a = &pa->e[k].act;
            if (u->player != maxplayer) continue;
            if (a->type == A_HARVEST || a->type == A_RETURN) r[1] += 1.0;
            if (a->type == A_PRODUCE) {
                if (a->utype == T_WORKER) r[2] += 1.0;
                else if (a->utype == T_BASE || a->utype == T_BARRACKS) r[3] += 1.0;
                else if (a->utype == T_LIGHT || a->utype == T_HEAVY || a->utype == T_RANGED) r[5] += 1.0;
            }
            if (a->type == A_ATTACK) r[4] += 1.0;
        }
    }
    if (gameover) r[0] = winner == maxplayer ? 1.0 : -1.0;
    for (int i = 0; i < 6; i++) d[i] = (uint8_t)(gameover ? 1 : 0);
}

/* PartiallyObservableGameState.observable(x, y) for `player`: some unit of the
 * player has sqrt(dx^2 + dy^2) <= sightRadius (README.md:90-92; UNPINNED,
 * DESIGN.md §4).                                                            */
static int observable(const OGS *g, int player, int x, int y) {
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!u->alive || u->player != player) continue;
        int dx = u->x - x, dy = u->y - y;
        if (dx * dx + dy * dy <= UT[u->type].sight * UT[u->type].sight) return 1;
    }
    return 0;
}

/* GameState.getVectorObservation(player).  With partial obs the observation is
 * that of new PartiallyObservableGameState(gs, player) -- every unit not owned
 * by the player (resources included) that the player cannot observe is
 * removed -- plus raw plane 6: the shown unit is observable by the opponent
 * (README.md:90-92 "visible to the opponent"; 0 on empty cells).            */
static void vector_obs(const OGS *g, int player, int partial, int32_t *raw) {
    int HW = g->W * g->H;
    int P = partial ? 7 : 6;
    memset(raw, 0, sizeof(int32_t) * P * HW);
    for (int c = 0; c < HW; c++) raw[5 * HW + c] = g->terrain[c];
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!u->alive) continue;
        if (partial && u->player != player && !observable(g, player, u->x, u->y)) continue;
        int c = u->y * g->W + u->x;
        if (partial) raw[6 * HW + c] = observable(g, 1 - player, u->x, u->y);
        raw[0 * HW + c] = u->hp;
        raw[1 * HW + c] = u->res;
        raw[2 * HW + c] = u->player < 0 ? 0 : (u->player == player ? 1 : 2);
        raw[3 * HW + c] = u->type + 1;
        raw[4 * HW + c] = u->assign >= 0 ? g->as[u->assign].act.type : A_NONE;
    }
}

/* JNIGridnetClient.getMasks(player) -> [HW][79] */
static void unit_masks(const OGS *g, int player, int32_t *m) {
    int HW = g->W * g->H;
    memset(m, 0, sizeof(int32_t) * HW * 79);
    OAct l[MAXLIST + 16];
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!u->alive || u->player != player || u->assign >= 0) continue;
        int32_t *v = m + 79 * (u->y * g->W + u->x);
        v[0] = 1;
        int n = unit_actions(g, i, 10, l);
        for (int k = 0; k < n; k++) { /* UnitAction.getValidActionArray, idxOffset 1 */
            const OAct *a = &l[k];
            v[1 + a->type] = 1;
            switch (a->type) {
            case A_MOVE: v[1 + 6 + a->param] = 1; break;
            case A_HARVEST: v[1 + 6 + 4 + a->param] = 1; break;
            case A_RETURN: v[1 + 6 + 8 + a->param] = 1; break;
            case A_PRODUCE:
                v[1 + 6 + 12 + a->param] = 1;
                v[1 + 6 + 16 + a->utype] = 1;
                break;
            case A_ATTACK: {
                int c = ATTACK_GRID / 2;
                int rx = a->x - u->x, ry = a->y - u->y;
                v[1 + 6 + 16 + NTYPES + (c + ry) * ATTACK_GRID + (c + rx)] = 1;
                break;
            }
            }
        }
    }
}

#include "mrts_oracle_ai.c"

/* ------------------------------------------------------------------------- */
OVec *ovec_create(int num_selfplay, int num_bot, int max_steps, int partial_obs, const OMap *maps,
                  int num_maps, const int32_t *game_map, const int32_t *bot_ai, const int32_t *bot_ai0) {
    OVec *v = (OVec *)calloc(1, sizeof(OVec));
    v->nsp = num_selfplay;
    v->nbot = num_bot;
    v->ngames = num_selfplay / 2 + num_bot;
    v->nenvs = num_selfplay + num_bot;
    v->max_steps = max_steps;
    v->partial_obs = partial_obs;
    v->nmaps = num_maps;
    v->maps = (OMap *)calloc(num_maps, sizeof(OMap));
    for (int i = 0; i < num_maps; i++) { /* deep copy */
        OMap *m = &v->maps[i];
        *m = maps[i];
        uint8_t *t = (uint8_t *)malloc(m->width * m->height);
        memcpy(t, maps[i].terrain, m->width * m->height);
        m->terrain = t;
        int32_t *u = (int32_t *)malloc(sizeof(int32_t) * 6 * (m->num_units + 1));
        memcpy(u, maps[i].units, sizeof(int32_t) * 6 * m->num_units);
        m->units = u;
    }
    v->W = maps[0].width;
    v->H = maps[0].height;
    v->game_map = (int *)calloc(v->ngames, sizeof(int));
    for (int i = 0; i < v->ngames; i++) v->game_map[i] = game_map ? game_map[i] : 0;
    v->bot_ai = (int *)calloc(num_bot + 1, sizeof(int));
    for (int i = 0; i < num_bot; i++) v->bot_ai[i] = bot_ai ? bot_ai[i] : OAI_PASSIVE;
    v->bot_ai0 = (int *)calloc(num_bot + 1, sizeof(int));
    for (int i = 0; i < num_bot; i++) v->bot_ai0[i] = bot_ai0 ? bot_ai0[i] : -1;
    v->gs = (OGS *)calloc(v->ngames, sizeof(OGS));
    v->env_steps = (int *)calloc(v->ngames, sizeof(int));
    v->ticks = (uint32_t *)calloc(v->ngames, sizeof(uint32_t));
    v->aam = (OAAMap *)calloc(2 * (size_t)v->ngames, sizeof(OAAMap)); /* [game][player] */
    v->raw = (int32_t *)calloc((size_t)v->nenvs * (partial_obs ? 7 : 6) * v->W * v->H, sizeof(int32_t));
    return v;
}

void ovec_destroy(OVec *v) {
    if (!v) return;
    for (int i = 0; i < v->ngames; i++) {
        free(v->gs[i].u);
        free(v->gs[i].as);
        free(v->gs[i].grid);
    }
    for (int i = 0; i < v->nmaps; i++) {
        free((void *)v->maps[i].terrain);
        free((void *)v->maps[i].units);
    }
    free(v->maps);
    free(v->game_map);
    free(v->bot_ai);
    free(v->bot_ai0);
    free(v->gs);
    free(v->env_steps);
    free(v->ticks);
    for (int i = 0; i < 2 * v->ngames; i++) free(v->aam[i].e);
    free(v->aam);
    free(v->raw);
    free(v);
}

int ovec_num_envs(const OVec *v) { return v->nenvs; }

/* env index -> (game, player): selfplay envs first (2k, 2k+1), then bot envs
 * (JNIGridnetVecClient ordering).                          */
static void env_views(const OVec *v, int game, int *env0, int *nviews) {
    if (game < v->nsp / 2) {
        *env0 = 2 * game;
        *nviews = 2;
    } else {
        *env0 = v->nsp + (game - v->nsp / 2);
        *nviews = 1;
    }
}

static void game_obs(OVec *v, int game) {
    int e0, nv;
    env_views(v, game, &e0, &nv);
    int P = v->partial_obs ? 7 : 6;
    size_t stride = (size_t)P * v->W * v->H;
    for (int k = 0; k < nv; k++) vector_obs(&v->gs[game], k, v->partial_obs, v->raw + (e0 + k) * stride);
}

void ovec_reset_game(OVec *v, int game, int map_id) {
    v->game_map[game] = map_id;
    gs_load(&v->gs[game], &v->maps[map_id]);
    v->env_steps[game] = 0;
    v->aam[2 * game].n = v->aam[2 * game + 1].n = 0; /* ai1/ai2.reset() */
    game_obs(v, game);
}

void ovec_event_counts(const OVec *v, int64_t *out) {
    for (int k = 0; k < OEV_N; k++) out[k] = 0;
    for (int g = 0; g < v->ngames; g++)
        for (int k = 0; k < OEV_N; k++) out[k] += v->gs[g].ev[k];
}

void ovec_reset(OVec *v) {
#pragma omp parallel for schedule(dynamic, 8)
    for (int g = 0; g < v->ngames; g++) ovec_reset_game(v, g, v->game_map[g]);
}

void ovec_get_masks(OVec *v, int32_t *masks) {
    size_t stride = (size_t)v->W * v->H * 79;
#pragma omp parallel for schedule(dynamic, 8)
    for (int g = 0; g < v->ngames; g++) {
        int e0, nv;
        env_views(v, g, &e0, &nv);
        for (int k = 0; k < nv; k++) unit_masks(&v->gs[g], k, masks + (e0 + k) * stride);
    }
}

void ovec_step(OVec *v, const int64_t *actions, const int32_t *src, double *reward, uint8_t *done) {
    int HW = v->W * v->H;
#pragma omp parallel for schedule(dynamic, 8)
    for (int gi = 0; gi < v->ngames; gi++) {
        OGS *g = &v->gs[gi];
        int e0, nv;
        env_views(v, gi, &e0, &nv);
        OPA pa0, pa1;
        if (nv == 2) { /* JNIGridnetClientSelfPlay.gameStep: p0 then p1 */
            jni_get_action(g, 0, actions + (size_t)e0 * HW * 7, src + (size_t)e0 * HW, &pa0);
            issue_safe(g, &pa0);
            jni_get_action(g, 1, actions + (size_t)(e0 + 1) * HW * 7, src + (size_t)(e0 + 1) * HW, &pa1);
            issue_safe(g, &pa1);
        } else { /* JNIGridnetClient.gameStep: both actions, then issue */
            const int b = gi - v->nsp / 2;
            if (v->bot_ai0[b] >= 0) /* JNIBotClient.gameStep: ai1.getAction(0), ai2.getAction(1) */
                bot_get_action(g, v->bot_ai0[b], 0, v->partial_obs, gi, v->ticks[gi], &v->aam[2 * gi], &pa0);
            else
                jni_get_action(g, 0, actions + (size_t)e0 * HW * 7, src + (size_t)e0 * HW, &pa0);
            bot_get_action(g, v->bot_ai[b], 1, v->partial_obs, gi, v->ticks[gi], &v->aam[2 * gi + 1], &pa1);
            issue_safe(g, &pa0);
            issue_safe(g, &pa1);
        }
        int gameover = cycle(g);
        int go2;
        int winner = gs_winner(g, &go2);
        for (int k = 0; k < nv; k++)
            rewards(g, &pa0, &pa1, k, gameover, winner, reward + 6 * (e0 + k), done + 6 * (e0 + k));
        pa_free(&pa0);
        pa_free(&pa1);
        v->env_steps[gi]++;
        v->ticks[gi]++;
        /* JNIGridnetVecClient.gameStep: done[0] || envSteps >= maxSteps -> reset,
         * keep the terminal reward/done and force done[0] = true.            */
        if (gameover || v->env_steps[gi] >= v->max_steps) {
            gs_load(g, &v->maps[v->game_map[gi]]);
            v->env_steps[gi] = 0;
            v->aam[2 * gi].n = v->aam[2 * gi + 1].n = 0;
            for (int k = 0; k < nv; k++) done[6 * (e0 + k)] = 1;
        }
        game_obs(v, gi);
    }
}

void ovec_raw_obs(OVec *v, int32_t *raw) {
    int P = v->partial_obs ? 7 : 6;
    memcpy(raw, v->raw, sizeof(int32_t) * (size_t)v->nenvs * P * v->W * v->H);
}

/* vec_env.py:311-321 */
void ovec_encode_obs(const int32_t *raw, int n, int h, int w, int partial_obs, int32_t *out) {
    static const int nplanes[7] = {5, 5, 3, 8, 6, 2, 2};
    int P_raw = partial_obs ? 7 : 6;
    int prefix[8] = {0};
    for (int i = 0; i < P_raw; i++) prefix[i + 1] = prefix[i] + nplanes[i];
    int P = prefix[P_raw];
    int HW = h * w;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < n; e++) {
        memset(out + (size_t)e * HW * P, 0, sizeof(int32_t) * (size_t)HW * P);
        for (int c = 0; c < HW; c++)
            for (int k = 0; k < P_raw; k++) {
                int val = raw[((size_t)e * P_raw + k) * HW + c];
                if (val < 0) val = 0;
                if (val > nplanes[k] - 1) val = nplanes[k] - 1;
                out[((size_t)e * HW + c) * P + prefix[k] + val] = 1;
            }
    }
}

int ovec_game_time(const OVec *v, int game) { return v->gs[game].time; }
void ovec_game_resources(const OVec *v, int game, int32_t *res2) {
    res2[0] = v->gs[game].res[0];
    res2[1] = v->gs[game].res[1];
}
void ovec_dump_cells(const OVec *v, int game, int32_t *out) {
    const OGS *g = &v->gs[game];
    int HW = g->W * g->H;
    for (int c = 0; c < HW; c++) {
        int32_t *o = out + 8 * c;
        int ui = g->grid[c];
        if (ui < 0) {
            o[0] = -1; o[1] = -1; o[2] = 0; o[3] = 0; o[4] = -1; o[5] = 0; o[6] = 0; o[7] = 0;
            continue;
        }
        const OUnit *u = &g->u[ui];
        o[0] = u->type; o[1] = u->player; o[2] = u->hp; o[3] = u->res;
        if (u->assign >= 0) {
            const OAssign *s = &g->as[u->assign];
            o[4] = s->act.type;
            o[5] = s->act.type == A_ATTACK ? (s->act.y * 1024 + s->act.x)
                   : s->act.type == A_PRODUCE ? s->act.param * 16 + s->act.utype
                                              : s->act.param;
            o[6] = s->time + eta(u, &s->act);
            o[7] = s->time;
        } else {
            o[4] = -1; o[5] = 0; o[6] = 0; o[7] = 0;
        }
    }
}

/* ---- Philox4x32-10 + masked sampler ------------------------------------- */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; i++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* one (env, cell) row of the masked sampler: m = the 78 channels */
static void sample_row(const int32_t *m, int e, int c, uint64_t seed, uint32_t step, int64_t *out) {
    static const int seg_off[7] = {0, 6, 10, 14, 18, 22, 29};
    static const int seg_len[7] = {6, 4, 4, 4, 4, 7, 49};
    uint32_t r[8];
    for (int h = 0; h < 2; h++) {
        uint32_t ctr[4] = {(uint32_t)c, (uint32_t)e, step, (uint32_t)h};
        philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (int j = 0; j < 4; j++) r[4 * h + j] = ctr[j];
    }
    for (int k = 0; k < 7; k++) {
        int nvalid = 0;
        for (int j = 0; j < seg_len[k]; j++) nvalid += m[seg_off[k] + j] != 0;
        int pick;
        if (nvalid == 0) {
            pick = (int)(((uint64_t)r[k] * (uint32_t)seg_len[k]) >> 32);
        } else {
            int t = (int)(((uint64_t)r[k] * (uint32_t)nvalid) >> 32);
            pick = 0;
            for (int j = 0; j < seg_len[k]; j++)
                if (m[seg_off[k] + j]) {
                    if (t == 0) { pick = j; break; }
                    t--;
                }
        }
        out[k] = pick;
    }
}

void ovec_sample_actions(const int32_t *m78, int n, int hw, int env0, uint64_t seed, uint32_t step, int64_t *act) {
#pragma omp parallel for schedule(static)
    for (int e = 0; e < n; e++)
        for (int c = 0; c < hw; c++)
            sample_row(m78 + ((size_t)e * hw + c) * 78, env0 + e, c, seed, step, act + ((size_t)e * hw + c) * 7);
}

/* The bench's CPU baseline: `steps` env-steps of every env -- getMasks, the
 * masked sampler on channels 1..78, gameStep, raw obs + one-hot encode -- with
 * OpenMP over games / envs and no Python between the stages.  Buffers are the
 * caller's: masks79 [N][HW][79], act [N][HW][7], src [N][HW], reward [N][6],
 * done [N][6], obs [N][HW][P]. */
void ovec_bench_steps(OVec *v, int steps, uint64_t seed, uint32_t step0, int32_t *masks79, int64_t *act, int32_t *src,
                      double *reward, uint8_t *done, int32_t *obs) {
    const int n = v->nenvs, hw = v->W * v->H;
    for (int s = 0; s < steps; s++) {
        ovec_get_masks(v, masks79);
#pragma omp parallel for schedule(static)
        for (int e = 0; e < n; e++)
            for (int c = 0; c < hw; c++) {
                const int32_t *m = masks79 + ((size_t)e * hw + c) * 79;
                src[(size_t)e * hw + c] = m[0];
                sample_row(m + 1, e, c, seed, step0 + (uint32_t)s, act + ((size_t)e * hw + c) * 7);
            }
        ovec_step(v, act, src, reward, done);
        ovec_encode_obs(v->raw, n, v->H, v->W, v->partial_obs, obs);
    }
}
