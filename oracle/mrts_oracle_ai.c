/*
 * mrts_oracle_ai.c -- CPU restatement of the scripted opponents of
 * gym_microrts/microrts_ai.py (/root/reference/gym_microrts/microrts_ai.py:1-61).
 * TEST INFRASTRUCTURE ONLY; #included by mrts_oracle.c (shares its types).
 *
 * The Java sources (ai.abstraction.{AbstractionLayerAI, WorkerRush, LightRush,
 * Move, Harvest, Attack, Train, Build}, ai.abstraction.partialobservability.PO*,
 * ai.abstraction.pathfinding.AStarPathFinding, ai.RandomBiasedAI, CoacAI in
 * lib/bots/Coac.jar) live in the absent submodule gym_microrts/microrts and the
 * absent jar; they are restated here from the public microRTS code base.  Bot
 * behaviour is therefore PARITY UNPINNED against Java (no fixture holds bot
 * decisions; the only outcome-level evidence is league.db); it
 * is pinned GPU == oracle bit for bit.  Restatement choices:
 *   - AStarPathFinding -> breadth-first distance from the goal set (free cells
 *     within range of the target); the first move goes to the start's free
 *     neighbour of least distance, ties UP, RIGHT, DOWN, LEFT.  Same path
 *     lengths and reachability as A*, A*'s open-list tie-break not kept.
 *   - AbstractionLayerAI.translateActions ends with fillWithNones(gs, p, 1).
 *   - RandomBiasedAI draws from a counter-based Philox stream keyed by
 *     (unit id, game tick, game) instead of an unseeded java.util.Random.
 *   - coacAI: CoacAI's strategy restated at the level of its published
 *     behaviour (coac_get_action), its free choices fixed by league.db's
 *     bot-vs-bot outcomes.
 *   - randomAI (RandomBiasedSingleUnitAI): one unit acting at a time.
 * The bot receives new PartiallyObservableGameState(gs, 1) under partial
 * observability (units it cannot observe are hidden), the full state otherwise,
 * and computes its PlayerAction before either player's actions of the tick are
 * issued (JNIGridnetClient.gameStep: ai1.getAction, ai2.getAction, issueSafe x2).
 */

static void philox(uint32_t c[4], uint32_t k0, uint32_t k1);

typedef struct {
    const OGS *g;
    int player;
    const uint8_t *hidden; /* per unit slot, NULL = full observability      */
    int partial;           /* gs instanceof PartiallyObservableGameState    */
} OView;

static int v_alive(const OView *v, int i) { return v->g->u[i].alive && !(v->hidden && v->hidden[i]); }
static int v_unit_at(const OView *v, int x, int y) { return unit_at_h(v->g, v->hidden, x, y); }
static int v_in(const OGS *g, int x, int y) { return x >= 0 && y >= 0 && x < g->W && y < g->H; }
static int v_free(const OView *v, int x, int y) { /* GameState.free */
    return v_in(v->g, x, y) && !terrain_at(v->g, x, y) && v_unit_at(v, x, y) < 0;
}
static int absi(int a) { return a < 0 ? -a : a; }

/* ---- ai.abstraction.AbstractAction and AbstractionLayerAI.actions ------- */
enum { AA_NONE = 0, AA_MOVE, AA_HARVEST, AA_ATTACK, AA_TRAIN, AA_BUILD };
typedef struct {
    int unit;      /* unit slot = Unit identity                               */
    int kind;
    int x, y;      /* Move / Build destination                                */
    int utype;     /* Train / Build unit type                                 */
    int target;    /* Harvest resource, Attack target (unit slots)            */
    int base;      /* Harvest stockpile (unit slot; may be dead: stale x, y)  */
    int completed; /* Train / Build                                           */
} OAA;
struct OAAMapS { /* LinkedHashMap<Unit, AbstractAction>: insertion order   */
    OAA *e;
    int n, cap;
};
typedef struct OAAMapS OAAMap;

static OAA *aa_get(OAAMap *m, int unit) {
    for (int k = 0; k < m->n; k++)
        if (m->e[k].unit == unit) return &m->e[k];
    return NULL;
}
static void aa_put(OAAMap *m, OAA a) { /* actions.put(u, aa): keeps the key's position */
    OAA *o = aa_get(m, a.unit);
    if (o) {
        *o = a;
        return;
    }
    if (m->n == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 32;
        m->e = (OAA *)xrealloc(m->e, sizeof(OAA) * m->cap);
    }
    m->e[m->n++] = a;
}
static OAA aa_new(int unit, int kind) {
    OAA a;
    memset(&a, 0, sizeof a);
    a.unit = unit;
    a.kind = kind;
    a.target = a.base = -1;
    return a;
}
static void ab_move(OAAMap *m, int u, int x, int y) { OAA a = aa_new(u, AA_MOVE); a.x = x; a.y = y; aa_put(m, a); }
static void ab_train(OAAMap *m, int u, int t) { OAA a = aa_new(u, AA_TRAIN); a.utype = t; aa_put(m, a); }
static void ab_build(OAAMap *m, int u, int t, int x, int y) {
    OAA a = aa_new(u, AA_BUILD);
    a.utype = t; a.x = x; a.y = y;
    aa_put(m, a);
}
static void ab_harvest(OAAMap *m, int u, int target, int base) {
    OAA a = aa_new(u, AA_HARVEST);
    a.target = target; a.base = base;
    aa_put(m, a);
}
static void ab_attack(OAAMap *m, int u, int target) { OAA a = aa_new(u, AA_ATTACK); a.target = target; aa_put(m, a); }

/* ---- AStarPathFinding.findPathToPositionInRange (restated, see header) ---- */
/* Returns the MOVE direction, or -1 for null (already within range, or no path). */
static int pf_dir(const OView *v, int ui, int tx, int ty, int range, const ORU *ru) {
    const OGS *g = v->g;
    const int W = g->W, H = g->H, HW = W * H, r2 = range * range;
    const OUnit *u = &g->u[ui];
    if ((u->x - tx) * (u->x - tx) + (u->y - ty) * (u->y - ty) <= r2) return -1;
    uint8_t fr[MAX_HW_ORACLE];
    int dist[MAX_HW_ORACLE], q[MAX_HW_ORACLE];
    for (int c = 0; c < HW; c++) fr[c] = (uint8_t)v_free(v, c % W, c / W);
    for (int i = 0; ru && i < ru->npos; i++)
        if (ru->pos[i] >= 0 && ru->pos[i] < HW) fr[ru->pos[i]] = 0;
    int qh = 0, qt = 0;
    for (int c = 0; c < HW; c++) {
        int dx = c % W - tx, dy = c / W - ty;
        dist[c] = -1;
        if (fr[c] && dx * dx + dy * dy <= r2) {
            dist[c] = 0;
            q[qt++] = c;
        }
    }
    while (qh < qt) {
        int c = q[qh++], x = c % W, y = c / W;
        const int nx[4] = {x, x + 1, x, x - 1}, ny[4] = {y - 1, y, y + 1, y};
        for (int d = 0; d < 4; d++) {
            if (!v_in(g, nx[d], ny[d])) continue;
            int n = ny[d] * W + nx[d];
            if (fr[n] && dist[n] < 0) {
                dist[n] = dist[c] + 1;
                q[qt++] = n;
            }
        }
    }
    int best = -1, bd = 0;
    const int sx[4] = {u->x, u->x + 1, u->x, u->x - 1}, sy[4] = {u->y - 1, u->y, u->y + 1, u->y};
    for (int d = 0; d < 4; d++) {
        if (!v_in(g, sx[d], sy[d])) continue;
        int n = sy[d] * W + sx[d];
        if (fr[n] && dist[n] >= 0 && (best < 0 || dist[n] < bd)) {
            best = d;
            bd = dist[n];
        }
    }
    return best;
}

/* GameState.isUnitActionAllowed(u, ua) on the bot's game state */
static int v_allowed(const OView *v, int ui, const OAct *a) {
    const OGS *g = v->g;
    const OUnit *u = &g->u[ui];
    if (a->type == A_MOVE) {
        int nx = u->x + (a->param == D_RIGHT) - (a->param == D_LEFT);
        int ny = u->y + (a->param == D_DOWN) - (a->param == D_UP);
        if (!v_free(v, nx, ny)) return 0;
    }
    ORU empty, r;
    ru_init(&empty);
    for (int i = 0; i < g->nu; i++) {
        if (!v_alive(v, i) || g->u[i].assign < 0) continue;
        resource_usage(g, &g->u[i], &g->as[g->u[i].assign].act, &r);
        ru_merge(&empty, &r);
        ru_free(&r);
    }
    resource_usage(g, u, a, &r);
    int ok = consistent_with(&r, &empty, g);
    ru_free(&r);
    ru_free(&empty);
    return ok;
}

static OAct mk(int type, int param, int utype) {
    OAct a = {type, param, 0, 0, utype};
    return a;
}
/* direction from (ux,uy) to the 4-adjacent (x,y), -1 when not adjacent */
static int adj_dir(int ux, int uy, int x, int y) {
    if (x == ux && y == uy - 1) return D_UP;
    if (x == ux + 1 && y == uy) return D_RIGHT;
    if (x == ux && y == uy + 1) return D_DOWN;
    if (x == ux - 1 && y == uy) return D_LEFT;
    return -1;
}

/* Train.score */
static int train_score(const OView *v, int x, int y, int type, int player) {
    const OGS *g = v->g;
    int dist = 0, first = 1;
    for (int i = 0; i < g->nu; i++) {
        if (!v_alive(v, i)) continue;
        const OUnit *o = &g->u[i];
        int want = UT[type].can_harvest ? UT[o->type].is_resource : (o->player >= 0 && o->player != player);
        if (!want) continue;
        int d = absi(o->x - x) + absi(o->y - y);
        if (first || d < dist) {
            dist = d;
            first = 0;
        }
    }
    return -dist;
}

static int aa_completed(const OView *v, const OAA *a) {
    const OUnit *u = &v->g->u[a->unit];
    switch (a->kind) {
    case AA_MOVE: return u->x == a->x && u->y == a->y;
    case AA_HARVEST:
    case AA_ATTACK: return !v_alive(v, a->target);
    default: return a->completed;
    }
}

/* AbstractAction.execute(gs, ru): 1 + *out, or 0 for null */
static int aa_execute(const OView *v, OAA *a, const ORU *ru, OAct *out) {
    const OGS *g = v->g;
    const OUnit *u = &g->u[a->unit];
    switch (a->kind) {
    case AA_MOVE: {
        int d = pf_dir(v, a->unit, a->x, a->y, 0, ru);
        if (d < 0) return 0;
        *out = mk(A_MOVE, d, -1);
        return v_allowed(v, a->unit, out);
    }
    case AA_HARVEST: {
        const OUnit *t = u->res == 0 ? &g->u[a->target] : &g->u[a->base];
        int d = pf_dir(v, a->unit, t->x, t->y, 1, ru);
        if (d >= 0) {
            *out = mk(A_MOVE, d, -1);
            return v_allowed(v, a->unit, out);
        }
        int ad = adj_dir(u->x, u->y, t->x, t->y);
        if (ad < 0) return 0;
        *out = mk(u->res == 0 ? A_HARVEST : A_RETURN, ad, -1);
        return 1;
    }
    case AA_ATTACK: {
        const OUnit *t = &g->u[a->target];
        int dx = t->x - u->x, dy = t->y - u->y, r = UT[u->type].range;
        if (dx * dx + dy * dy <= r * r) {
            OAct at = {A_ATTACK, DIRECTION_NONE, t->x, t->y, -1};
            *out = at;
            return 1;
        }
        int d = pf_dir(v, a->unit, t->x, t->y, r, ru);
        if (d < 0) return 0;
        *out = mk(A_MOVE, d, -1);
        return v_allowed(v, a->unit, out);
    }
    case AA_TRAIN: {
        int best = -1, bs = -1;
        const int nx[4] = {u->x, u->x + 1, u->x, u->x - 1}, ny[4] = {u->y - 1, u->y, u->y + 1, u->y};
        for (int d = 0; d < 4; d++) {
            if (!v_free(v, nx[d], ny[d])) continue;
            int sc = train_score(v, nx[d], ny[d], a->utype, u->player);
            if (sc > bs || best == -1) {
                bs = sc;
                best = d;
            }
        }
        a->completed = 1;
        if (best < 0) return 0;
        *out = mk(A_PRODUCE, best, a->utype);
        return v_allowed(v, a->unit, out);
    }
    case AA_BUILD: {
        int d = pf_dir(v, a->unit, a->x, a->y, 1, ru);
        if (d >= 0) {
            *out = mk(A_MOVE, d, -1);
            return v_allowed(v, a->unit, out);
        }
        int ad = adj_dir(u->x, u->y, a->x, a->y);
        if (ad < 0) return 0;
        *out = mk(A_PRODUCE, ad, a->utype);
        if (!v_allowed(v, a->unit, out)) return 0;
        a->completed = 1;
        return 1;
    }
    }
    return 0;
}

static void fill_with_nones(const OGS *g, int player, OPA *pa, int duration) { /* PlayerAction.fillWithNones */
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!u->alive || u->player != player || u->assign >= 0) continue;
        int found = 0;
        for (int k = 0; k < pa->n && !found; k++) found = pa->e[k].unit == i;
        if (!found) {
            OAct a = act_none(duration);
            pa_add(pa, i, &a);
        }
    }
}

/* AbstractionLayerAI.translateActions */
static void translate_actions(const OView *v, OAAMap *m, OPA *pa) {
    const OGS *g = v->g;
    pa_init(pa);
    int w = 0;
    for (int k = 0; k < m->n; k++) {
        OAA *a = &m->e[k];
        int del = !v_alive(v, a->unit) || aa_completed(v, a);
        if (!del && g->u[a->unit].assign < 0) {
            OAct ua;
            if (aa_execute(v, a, &pa->ru, &ua)) {
                ORU r;
                resource_usage(g, &g->u[a->unit], &ua, &r);
                if (consistent_with(&r, &pa->ru, g)) {
                    ru_merge(&pa->ru, &r);
                    pa_add(pa, a->unit, &ua);
                }
                ru_free(&r);
            }
        }
        if (!del) m->e[w++] = *a; /* toDelete removed after the loop, order kept */
    }
    m->n = w;
    fill_with_nones(g, v->player, pa, 1);
}

/* ---- shared behaviours ---------------------------------------------------- */
static int closest_enemy(const OView *v, int ui) {
    const OGS *g = v->g;
    const OUnit *u = &g->u[ui];
    int best = -1, bd = 0;
    for (int i = 0; i < g->nu; i++) {
        if (!v_alive(v, i)) continue;
        const OUnit *o = &g->u[i];
        if (o->player < 0 || o->player == u->player) continue;
        int d = absi(o->x - u->x) + absi(o->y - u->y);
        if (best < 0 || d < bd) {
            best = i;
            bd = d;
        }
    }
    return best;
}
static int closest_of(const OView *v, int ui, int want_resource) { /* resource, or own stockpile */
    const OGS *g = v->g;
    const OUnit *u = &g->u[ui];
    int best = -1, bd = 0;
    for (int i = 0; i < g->nu; i++) {
        if (!v_alive(v, i)) continue;
        const OUnit *o = &g->u[i];
        int ok = want_resource ? UT[o->type].is_resource : (UT[o->type].is_stockpile && o->player == u->player);
        if (!ok) continue;
        int d = absi(o->x - u->x) + absi(o->y - u->y);
        if (best < 0 || d < bd) {
            best = i;
            bd = d;
        }
    }
    return best;
}

/* meleeUnitBehavior (+ the exploration of the PO* rushes when nothing is seen) */
static void melee_behavior(const OView *v, OAAMap *m, int ui, int po) {
    const OGS *g = v->g;
    int e = closest_enemy(v, ui);
    if (e >= 0) {
        ab_attack(m, ui, e);
        return;
    }
    if (!(po && v->partial)) return;
    const OUnit *u = &g->u[ui];
    int cx = 0, cy = 0, cd = -1;
    for (int y = 0; y < g->H; y++)
        for (int x = 0; x < g->W; x++) {
            if (observable(g, v->player, x, y)) continue;
            int d = (u->x - x) * (u->x - x) + (u->y - y) * (u->y - y);
            if (cd == -1 || d < cd) {
                cx = x; cy = y; cd = d;
            }
        }
    if (cd != -1) ab_move(m, ui, cx, cy);
}

/* harvest(u, closest resource, closest base) unless already harvesting those */
static void harvest_behavior(const OView *v, OAAMap *m, int ui) {
    int r = closest_of(v, ui, 1), b = closest_of(v, ui, 0);
    if (r < 0 || b < 0) return;
    OAA *a = aa_get(m, ui);
    if (a && a->kind == AA_HARVEST && a->target == r && a->base == b) return;
    ab_harvest(m, ui, r, b);
}

/* AbstractionLayerAI.findBuildingPosition */
static int find_building_position(const OView *v, const int *reserved, int nres, int dx, int dy) {
    const OGS *g = v->g;
    const int W = g->W, H = g->H, L = W > H ? W : H;
    for (int l = 1; l < L; l++) {
        for (int side = 0; side < 4; side++) {
            for (int k = -l; k <= l; k++) {
                int x, y;
                if (side == 0) { y = dy - l; x = dx + k; if (y < 0) break; }
                else if (side == 1) { x = dx + l; y = dy + k; if (x >= W) break; }
                else if (side == 2) { y = dy + l; x = dx + k; if (y >= H) break; }
                else { x = dx - l; y = dy + k; if (x < 0) break; }
                if (x < 0 || y < 0 || x >= W || y >= H) continue;
                int pos = x + y * W, taken = 0;
                for (int i = 0; i < nres; i++) taken |= reserved[i] == pos;
                if (!taken && v_free(v, x, y)) return pos;
            }
        }
    }
    return -1;
}

static void build_if_not_already(const OView *v, OAAMap *m, int ui, int type, int *reserved, int *nres) {
    OAA *a = aa_get(m, ui);
    if (a && a->kind == AA_BUILD && a->utype == type) return;
    const OUnit *u = &v->g->u[ui];
    int pos = find_building_position(v, reserved, *nres, u->x, u->y);
    ab_build(m, ui, type, pos % v->g->W, pos / v->g->W); /* Java int division: -1 -> (-1, 0) */
    reserved[(*nres)++] = pos;
}

static int count_own(const OView *v, int type) {
    int n = 0;
    for (int i = 0; i < v->g->nu; i++) n += v_alive(v, i) && v->g->u[i].type == type && v->g->u[i].player == v->player;
    return n;
}
static int count_enemy(const OView *v, int type) {
    int n = 0;
    for (int i = 0; i < v->g->nu; i++)
        n += v_alive(v, i) && v->g->u[i].type == type && v->g->u[i].player >= 0 && v->g->u[i].player != v->player;
    return n;
}

/* ---- WorkerRush / LightRush / HeavyRush / RangedRush (+ PO* variants) ---- */
/* army == T_WORKER: WorkerRush; otherwise the barracks unit of the rush. */
static void rush_get_action(const OView *v, OAAMap *m, int army, int po, int coac, OPA *pa) {
    const OGS *g = v->g;
    const int p = v->player;
    const int res = g->res[p];
    int nworkers = count_own(v, T_WORKER), nbases = count_own(v, T_BASE), nbarracks = count_own(v, T_BARRACKS);
    /* bases */
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || u->type != T_BASE || u->player != p || u->assign >= 0) continue;
        if (army == T_WORKER) {
            if (res >= UT[T_WORKER].cost) ab_train(m, i, T_WORKER);
        } else if (coac) {
            if (nworkers < 2 * nbases + 2 && res >= UT[T_WORKER].cost) ab_train(m, i, T_WORKER);
        } else if (nworkers < 1 && res >= UT[T_WORKER].cost) {
            ab_train(m, i, T_WORKER);
        }
    }
    /* barracks */
    if (army != T_WORKER) {
        int t = army;
        if (coac) /* ranged by default; heavies against light-heavy armies */
            t = count_enemy(v, T_LIGHT) > count_enemy(v, T_RANGED) + count_enemy(v, T_HEAVY) ? T_HEAVY : T_RANGED;
        for (int i = 0; i < g->nu; i++) {
            const OUnit *u = &g->u[i];
            if (!v_alive(v, i) || u->type != T_BARRACKS || u->player != p || u->assign >= 0) continue;
            if (res >= UT[t].cost) ab_train(m, i, t);
        }
    }
    /* melee units */
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || !UT[u->type].can_attack || UT[u->type].can_harvest || u->player != p || u->assign >= 0)
            continue;
        melee_behavior(v, m, i, po);
    }
    /* workers (busy ones included) */
    int free_w[MAX_HW_ORACLE], nf = 0;
    for (int i = 0; i < g->nu; i++)
        if (v_alive(v, i) && UT[g->u[i].type].can_harvest && g->u[i].player == p) free_w[nf++] = i;
    if (nf == 0) {
        translate_actions(v, m, pa);
        return;
    }
    int reserved[8], nres = 0, used = 0, head = 0;
    if (nbases == 0 && head < nf && res >= UT[T_BASE].cost + used) {
        build_if_not_already(v, m, free_w[head++], T_BASE, reserved, &nres);
        used += UT[T_BASE].cost;
    }
    if (army == T_WORKER) {
        if (head < nf) harvest_behavior(v, m, free_w[head++]);
        for (int k = head; k < nf; k++) melee_behavior(v, m, free_w[k], po);
    } else {
        if (nbarracks == 0 && res >= UT[T_BARRACKS].cost + used && head < nf) {
            build_if_not_already(v, m, free_w[head++], T_BARRACKS, reserved, &nres);
            used += UT[T_BARRACKS].cost;
        }
        if (coac) {
            int nh = 2 * (nbases > 0 ? nbases : 1);
            for (int k = head; k < nf; k++) {
                if (k - head < nh) harvest_behavior(v, m, free_w[k]);
                else melee_behavior(v, m, free_w[k], po);
            }
        } else {
            for (int k = head; k < nf; k++) harvest_behavior(v, m, free_w[k]);
        }
    }
    translate_actions(v, m, pa);
}


/* ---- coacAI ------------------------------------------------------------------
 * CoacAI (Coac.jar, vec_env.py:158; microrts_ai.py:58-61) restated at the level
 * of its published strategy -- the jar is absent, so this is PARITY UNPINNED
 * against Java and pinned only at the outcome level: the free choices below
 * were fixed so that every bot-vs-bot outcome league.db records on
 * basesWorkers16x16A (tests/golden/league_outcomes.json) is reproduced
 * (DESIGN.md §4b):
 *   - economy: each idle base trains a worker while the player owns fewer than
 *     2 * bases + 2 workers; the first 2 * max(bases, 1) workers of the unit
 *     list harvest (closest resource / closest base);
 *   - one barracks, built once the player owns >= 2 workers (after a base
 *     rebuild when no base is left); it trains ranged units, heavies when the
 *     enemy fields more light units than ranged + heavy;
 *   - army units attack the closest enemy;
 *   - the remaining workers defend: attack the closest enemy when it is within
 *     Manhattan distance 8 of the worker's closest own base, harvest otherwise. */
enum { COAC_HARVESTERS_PER_BASE = 2, COAC_EXTRA_WORKERS = 2, COAC_BARRACKS_MIN_WORKERS = 2, COAC_DEFENSE_RADIUS = 8 };
static int manh(const OUnit *a, const OUnit *b) { return absi(a->x - b->x) + absi(a->y - b->y); }
static void coac_get_action(const OView *v, OAAMap *m, OPA *pa) {
    const OGS *g = v->g;
    const int p = v->player;
    const int res = g->res[p];
    int nworkers = count_own(v, T_WORKER), nbases = count_own(v, T_BASE), nbarracks = count_own(v, T_BARRACKS);
    for (int i = 0; i < g->nu; i++) { /* bases */
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || u->type != T_BASE || u->player != p || u->assign >= 0) continue;
        if (nworkers < COAC_HARVESTERS_PER_BASE * nbases + COAC_EXTRA_WORKERS && res >= UT[T_WORKER].cost)
            ab_train(m, i, T_WORKER);
    }
    const int t = count_enemy(v, T_LIGHT) > count_enemy(v, T_RANGED) + count_enemy(v, T_HEAVY) ? T_HEAVY : T_RANGED;
    for (int i = 0; i < g->nu; i++) { /* barracks */
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || u->type != T_BARRACKS || u->player != p || u->assign >= 0) continue;
        if (res >= UT[t].cost) ab_train(m, i, t);
    }
    for (int i = 0; i < g->nu; i++) { /* army */
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || !UT[u->type].can_attack || UT[u->type].can_harvest || u->player != p || u->assign >= 0)
            continue;
        melee_behavior(v, m, i, 0);
    }
    int free_w[MAX_HW_ORACLE], nf = 0; /* workers, busy ones included */
    for (int i = 0; i < g->nu; i++)
        if (v_alive(v, i) && UT[g->u[i].type].can_harvest && g->u[i].player == p) free_w[nf++] = i;
    int reserved[8], nres = 0, used = 0, head = 0;
    if (nbases == 0 && head < nf && res >= UT[T_BASE].cost + used) {
        build_if_not_already(v, m, free_w[head++], T_BASE, reserved, &nres);
        used += UT[T_BASE].cost;
    }
    if (nbarracks == 0 && res >= UT[T_BARRACKS].cost + used && head < nf && nworkers >= COAC_BARRACKS_MIN_WORKERS) {
        build_if_not_already(v, m, free_w[head++], T_BARRACKS, reserved, &nres);
        used += UT[T_BARRACKS].cost;
    }
    const int nh = COAC_HARVESTERS_PER_BASE * (nbases > 0 ? nbases : 1);
    for (int k = head; k < nf; k++) {
        const int w = free_w[k];
        if (k - head < nh) {
            harvest_behavior(v, m, w);
            continue;
        }
        const int e = closest_enemy(v, w), b = closest_of(v, w, 0);
        if (e < 0) continue;
        if (b < 0 || manh(&g->u[b], &g->u[e]) <= COAC_DEFENSE_RADIUS) ab_attack(m, w, e);
        else harvest_behavior(v, m, w);
    }
    translate_actions(v, m, pa);
}

/* ---- RandomBiasedAI.getAction --------------------------------------------- */
static void random_biased_get_action(const OView *v, int game, uint32_t tick, OPA *pa) {
    /* stream per (unit, tick, game, player); player 1 keeps the 'RAND' tag */
    const uint32_t tag = 0x52414E44u + (uint32_t)(1 - v->player);
    const OGS *g = v->g;
    const int p = v->player;
    pa_init(pa);
    ORU r;
    for (int i = 0; i < g->nu; i++) { /* reserved resources of the pending assignments */
        if (!v_alive(v, i) || g->u[i].assign < 0) continue;
        resource_usage(g, &g->u[i], &g->as[g->u[i].assign].act, &r);
        ru_merge(&pa->ru, &r);
        ru_free(&r);
    }
    OAct l[MAXLIST + 16];
    for (int i = 0; i < g->nu; i++) {
        const OUnit *u = &g->u[i];
        if (!v_alive(v, i) || u->player != p || u->assign >= 0) continue;
        int n = unit_actions_h(g, v->hidden, i, 10, l);
        int total = 0;
        for (int k = 0; k < n; k++)
            total += (l[k].type == A_ATTACK || l[k].type == A_HARVEST || l[k].type == A_RETURN) ? 5 : 1;
        uint32_t ctr[4] = {(uint32_t)i, tick, (uint32_t)game, tag};
        philox(ctr, 0x5EED5EEDu, 0xB0B0B0B0u);
        int t = (int)(((uint64_t)ctr[0] * (uint32_t)total) >> 32), pick = n - 1;
        for (int k = 0; k < n; k++) {
            t -= (l[k].type == A_ATTACK || l[k].type == A_HARVEST || l[k].type == A_RETURN) ? 5 : 1;
            if (t < 0) {
                pick = k;
                break;
            }
        }
        resource_usage(g, u, &l[pick], &r);
        if (consistent_with(&r, &pa->ru, g)) {
            ru_merge(&pa->ru, &r);
            pa_add(pa, i, &l[pick]);
        } else {
            pa_add(pa, i, &l[n - 1]); /* the NONE(10) of the list */
        }
        ru_free(&r);
    }
}

/* ---- RandomBiasedSingleUnitAI (randomAI, microrts_ai.py:7-10) --------------------
 * One unit acts at a time: while any unit of the player holds an action
 * assignment the AI returns an empty PlayerAction; otherwise one idle unit,
 * drawn uniformly, gets an action of getUnitActions(gs, 10) drawn with
 * RandomBiasedAI's weights (5 for attack / harvest / return, 1 otherwise; the
 * NONE(10) of the list when inconsistent).  Unseeded java.util.Random in Java;
 * here Philox keyed by (tick, game) like randomBiasedAI.  Outcome-pinned by
 * league.db (randomAI draws vs passiveAI, loses to every other bot). */
static void random_single_get_action(const OView *v, int game, uint32_t tick, OPA *pa) {
    const OGS *g = v->g;
    const int p = v->player;
    pa_init(pa);
    int idle[MAX_HW_ORACLE], ni = 0;
    for (int i = 0; i < g->nu; i++) {
        if (!v_alive(v, i) || g->u[i].player != p) continue;
        if (g->u[i].assign >= 0) return; /* a unit is still busy */
        idle[ni++] = i;
    }
    if (ni == 0) return;
    ORU r;
    for (int i = 0; i < g->nu; i++) { /* reserved resources of the pending assignments */
        if (!v_alive(v, i) || g->u[i].assign < 0) continue;
        resource_usage(g, &g->u[i], &g->as[g->u[i].assign].act, &r);
        ru_merge(&pa->ru, &r);
        ru_free(&r);
    }
    uint32_t ctr[4] = {0xFFFFFFFFu, tick, (uint32_t)game, 0x52534E47u + (uint32_t)(1 - p)};
    philox(ctr, 0x5EED5EEDu, 0xB0B0B0B0u);
    const int i = idle[(int)(((uint64_t)ctr[1] * (uint32_t)ni) >> 32)];
    OAct l[MAXLIST + 16];
    const int n = unit_actions_h(g, v->hidden, i, 10, l);
    int total = 0;
    for (int k = 0; k < n; k++) total += (l[k].type == A_ATTACK || l[k].type == A_HARVEST || l[k].type == A_RETURN) ? 5 : 1;
    int t = (int)(((uint64_t)ctr[0] * (uint32_t)total) >> 32), pick = n - 1;
    for (int k = 0; k < n; k++) {
        t -= (l[k].type == A_ATTACK || l[k].type == A_HARVEST || l[k].type == A_RETURN) ? 5 : 1;
        if (t < 0) {
            pick = k;
            break;
        }
    }
    resource_usage(g, &g->u[i], &l[pick], &r);
    if (consistent_with(&r, &pa->ru, g)) pa_add(pa, i, &l[pick]);
    else pa_add(pa, i, &l[n - 1]);
    ru_free(&r);
}

/* ai.getAction(player, gs) for a bot game: ai2 for player 1 (bot envs), and
 * ai1 for player 0 in bot-vs-bot games (MicroRTSBotVecEnv, vec_env.py:1104-1236) */
static void bot_get_action(const OGS *g, int ai, int player, int partial, int game, uint32_t tick, OAAMap *m, OPA *pa) {
    uint8_t *hidden = NULL;
    if (partial) {
        hidden = (uint8_t *)calloc(g->nu + 1, 1);
        for (int i = 0; i < g->nu; i++)
            if (g->u[i].alive && g->u[i].player != player) hidden[i] = !observable(g, player, g->u[i].x, g->u[i].y);
    }
    OView v = {g, player, hidden, partial};
    switch (ai) {
    case OAI_WORKER_RUSH: rush_get_action(&v, m, T_WORKER, 0, 0, pa); break;
    case OAI_LIGHT_RUSH: rush_get_action(&v, m, T_LIGHT, 0, 0, pa); break;
    case OAI_PO_WORKER_RUSH: rush_get_action(&v, m, T_WORKER, 1, 0, pa); break;
    case OAI_PO_LIGHT_RUSH: rush_get_action(&v, m, T_LIGHT, 1, 0, pa); break;
    case OAI_PO_HEAVY_RUSH: rush_get_action(&v, m, T_HEAVY, 1, 0, pa); break;
    case OAI_PO_RANGED_RUSH: rush_get_action(&v, m, T_RANGED, 1, 0, pa); break;
    case OAI_COAC: coac_get_action(&v, m, pa); break;
    case OAI_RANDOM_BIASED: random_biased_get_action(&v, game, tick, pa); break;
    case OAI_RANDOM: random_single_get_action(&v, game, tick, pa); break;
    default: passive_get_action((OGS *)g, player, pa); break;
    }
    free(hidden);
}
