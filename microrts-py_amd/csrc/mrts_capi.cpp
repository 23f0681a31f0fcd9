// mrts_capi.cpp -- C ABI of libmicrorts_amd.so (include/microrts_amd.h).
//
// Host side of the replacement for tests.JNIGridnetVecClient
// (/root/reference/gym_microrts/envs/vec_env.py:256-276): config validation,
// PhysicalGameState XML loading into device map templates, workspace carving
// and kernel dispatch.  No torch types cross this boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "microrts_amd.h"
#include "mrts_engine.h"
#include "mrts_layout.h"

namespace {

const char *kTypeNames[MRTS_NTYPES] = {"Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"};

struct MapData {
    int w = 0, h = 0;
    std::vector<uint8_t> wall;
    int res[2] = {0, 0};
    std::vector<int4> cells;  // template records (unit word, uid, 0, 0)
    int nunits = 0;
};

std::string attr(const std::string &tag, const char *name) {
    std::string key = std::string(" ") + name + "=\"";
    size_t p = tag.find(key);
    if (p == std::string::npos) return std::string();
    p += key.size();
    size_t q = tag.find('"', p);
    return q == std::string::npos ? std::string() : tag.substr(p, q - p);
}

bool to_int(const std::string &s, int *out) {
    if (s.empty()) return false;
    char *end = nullptr;
    long v = std::strtol(s.c_str(), &end, 10);
    if (*end) return false;
    *out = (int)v;
    return true;
}

uint32_t unit_word(int type, int owner, int hp, int res) {
    return (uint32_t)(type + 1) | ((uint32_t)(owner + 1) << 4) | ((uint32_t)hp << 6) | ((uint32_t)res << 16);
}

// rts.PhysicalGameState.load (XML form of /root/reference/PCG/maps/wall-1:1-16)
bool load_map(const char *path, MapData *m, std::string *err) {
    std::ifstream f(path);
    if (!f) { *err = std::string("cannot open map ") + path; return false; }
    std::stringstream ss;
    ss << f.rdbuf();
    std::string x = ss.str();
    size_t root = x.find("<rts.PhysicalGameState");
    if (root == std::string::npos) { *err = std::string("not a PhysicalGameState XML: ") + path; return false; }
    std::string rtag = x.substr(root, x.find('>', root) - root);
    if (!to_int(attr(rtag, "width"), &m->w) || !to_int(attr(rtag, "height"), &m->h) || m->w <= 0 || m->h <= 0) {
        *err = std::string("bad width/height in ") + path;
        return false;
    }
    const int HW = m->w * m->h;
    if (HW > MRTS_MAX_HW) { *err = "map larger than MRTS_MAX_HW cells"; return false; }
    size_t t0 = x.find("<terrain>"), t1 = x.find("</terrain>");
    if (t0 == std::string::npos || t1 == std::string::npos) { *err = "missing <terrain>"; return false; }
    std::string terr;
    for (size_t i = t0 + 9; i < t1; i++)
        if (x[i] == '0' || x[i] == '1') terr.push_back(x[i]);
    if ((int)terr.size() != HW) { *err = std::string("terrain length mismatch in ") + path; return false; }
    m->wall.assign(HW, 0);
    for (int i = 0; i < HW; i++) m->wall[i] = terr[i] == '1';
    size_t pos = 0;
    while ((pos = x.find("<rts.Player ", pos)) != std::string::npos) {
        std::string tag = x.substr(pos, x.find('>', pos) - pos);
        int id = -1, r = 0;
        if (!to_int(attr(tag, "ID"), &id) || !to_int(attr(tag, "resources"), &r) || id < 0 || id > 1) {
            *err = "bad <rts.Player>";
            return false;
        }
        m->res[id] = r;
        pos += 12;
    }
    m->cells.assign(HW, make_int4(0, 0, 0, 0));
    pos = 0;
    int idx = 0;
    while ((pos = x.find("<rts.units.Unit ", pos)) != std::string::npos) {
        std::string tag = x.substr(pos, x.find('>', pos) - pos);
        std::string tn = attr(tag, "type");
        int type = -1;
        for (int k = 0; k < MRTS_NTYPES; k++)
            if (tn == kTypeNames[k]) type = k;
        int player, ux, uy, ur, hp;
        if (type < 0 || !to_int(attr(tag, "player"), &player) || !to_int(attr(tag, "x"), &ux) ||
            !to_int(attr(tag, "y"), &uy) || !to_int(attr(tag, "resources"), &ur) || !to_int(attr(tag, "hitpoints"), &hp)) {
            *err = std::string("bad <rts.units.Unit> in ") + path;
            return false;
        }
        if (ux < 0 || uy < 0 || ux >= m->w || uy >= m->h || player < -1 || player > 1 || hp < 1 || hp > 1023 ||
            ur < 0 || ur > 65535) {
            *err = std::string("unit out of range in ") + path;
            return false;
        }
        int c = uy * m->w + ux;
        if (m->cells[c].x != 0) { *err = std::string("two units in one cell in ") + path; return false; }
        m->cells[c] = make_int4((int)unit_word(type, player, hp, ur), idx++, 0, 0);
        pos += 16;
    }
    m->nunits = idx;
    return true;
}

std::string utt_json() {
    // rts.units.UnitTypeTable.toJSON of UnitTypeTable() (VERSION_ORIGINAL)
    struct T { const char *n; int cost, hp, mind, maxd, range, pt, mt, at, ht, rt, ha, sight; int res, stock, harv, move, atk; const char *prod, *by; };
    static const T ts[] = {
        {"Resource", 1, 1, 1, 1, 1, 10, 10, 10, 10, 10, 1, 0, 1, 0, 0, 0, 0, "", ""},
        {"Base", 10, 10, 1, 1, 1, 250, 10, 10, 10, 10, 1, 5, 0, 1, 0, 0, 0, "\"Worker\"", "\"Worker\""},
        {"Barracks", 5, 4, 1, 1, 1, 200, 10, 10, 10, 10, 1, 3, 0, 0, 0, 0, 0, "\"Light\", \"Heavy\", \"Ranged\"", "\"Worker\""},
        {"Worker", 1, 1, 1, 1, 1, 50, 10, 5, 20, 10, 1, 3, 0, 0, 1, 1, 1, "\"Base\", \"Barracks\"", "\"Base\""},
        {"Light", 2, 4, 2, 2, 1, 80, 8, 5, 10, 10, 1, 2, 0, 0, 0, 1, 1, "", "\"Barracks\""},
        {"Heavy", 2, 4, 4, 4, 1, 120, 12, 5, 10, 10, 1, 2, 0, 0, 0, 1, 1, "", "\"Barracks\""},
        {"Ranged", 2, 1, 1, 1, 3, 100, 10, 5, 10, 10, 1, 3, 0, 0, 0, 1, 1, "", "\"Barracks\""},
    };
    std::string s = "{\"moveConflictResolutionStrategy\":3,\"unitTypes\":[";
    char buf[1024];
    for (int i = 0; i < MRTS_NTYPES; i++) {
        const T &t = ts[i];
        std::snprintf(buf, sizeof buf,
                      "%s{\"ID\":%d, \"name\":\"%s\", \"cost\":%d, \"hp\":%d, \"minDamage\":%d, \"maxDamage\":%d, "
                      "\"attackRange\":%d, \"produceTime\":%d, \"moveTime\":%d, \"attackTime\":%d, \"harvestTime\":%d, "
                      "\"returnTime\":%d, \"harvestAmount\":%d, \"sightRadius\":%d, \"isResource\":%s, \"isStockpile\":%s, "
                      "\"canHarvest\":%s, \"canMove\":%s, \"canAttack\":%s, \"produces\":[%s], \"producedBy\":[%s]}",
                      i ? ", " : "", i, t.n, t.cost, t.hp, t.mind, t.maxd, t.range, t.pt, t.mt, t.at, t.ht, t.rt, t.ha,
                      t.sight, t.res ? "true" : "false", t.stock ? "true" : "false", t.harv ? "true" : "false",
                      t.move ? "true" : "false", t.atk ? "true" : "false", t.prod, t.by);
        s += buf;
    }
    s += "]}";
    return s;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// int4 records between consecutive games' cell rows (a padded stride measured
// neutral, profiles/r04_ab/README.md)
int cell_stride(int HW) { return HW; }

}  // namespace

struct mrts_vec {
    int nsp = 0, nbot = 0, ngames = 0, nenvs = 0, max_steps = 0, partial_obs = 0, obs_float = 0;
    int W = 0, H = 0, HW = 0;
    std::vector<MapData> maps;
    std::vector<std::string> map_path;   // as given to mrts_create / mrts_add_map
    int map_capacity = 0;                // map template slots carved in the workspace
    std::vector<int32_t> game_map;
    std::vector<int32_t> bot_ai;
    std::vector<int32_t> bot_ai0;   // -1: the agent plays player 0
    int nbot0 = 0;
    int game_offset = 0;
    // workspace carving
    size_t off_cells = 0, off_genv = 0, off_mcells = 0, off_mwall = 0, off_mscal = 0, off_scratch = 0, total = 0;
    size_t off_botai = 0, off_botai0 = 0, off_aa = 0, off_botpa = 0, off_parked = 0;
    std::vector<uint8_t> parked;   // host mirror of the device parked flags (mrts_park_games)
    int nbot_active = 0;
    unsigned char *ws = nullptr;
    std::vector<int32_t> scratch_host;
    std::string err, utt;
    double rw[6] = {0, 0, 0, 0, 0, 0};
    int shaping = 1;
    int32_t *next_mask = nullptr, *next_src = nullptr;   // mrts_bind_mask_outputs
    EngineParams base{};
    // bot fusion (mrts_set_bot_fusion): k_step decides the next tick's bot actions
    int fuse = 1;             // requested
    bool bots_ready = false;  // the bot decisions for the current state are in botpa / aa
};

static int fail(mrts_vec *h, int code, const std::string &msg) {
    if (h) h->err = msg;
    return code;
}
static int hip_fail(mrts_vec *h, hipError_t e, const char *what) {
    return fail(h, MRTS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

extern "C" {

const char *mrts_version(void) { return "microrts_amd 0.1 (gfx950)"; }

int mrts_create(const mrts_config *cfg, mrts_vec **out) {
    if (!cfg || !out) return MRTS_EINVAL;
    *out = nullptr;
    mrts_vec *h = new mrts_vec();
    h->utt = utt_json();
    *out = h;
    if (cfg->num_selfplay_envs < 0 || cfg->num_bot_envs < 0 || (cfg->num_selfplay_envs & 1))
        return fail(h, MRTS_EINVAL, "num_selfplay_envs must be even and >= 0, num_bot_envs >= 0");
    if (cfg->num_selfplay_envs + cfg->num_bot_envs <= 0) return fail(h, MRTS_EINVAL, "no envs");
    if (cfg->max_steps <= 0 || cfg->max_steps >= MRTS_MAX_TIME)
        return fail(h, MRTS_EINVAL, "max_steps must be in [1, 500000)");
    if (cfg->num_maps <= 0 || !cfg->map_paths) return fail(h, MRTS_EINVAL, "no maps");
    h->nsp = cfg->num_selfplay_envs;
    h->nbot = cfg->num_bot_envs;
    h->ngames = h->nsp / 2 + h->nbot;
    h->nenvs = h->nsp + h->nbot;
    h->max_steps = cfg->max_steps;
    h->partial_obs = cfg->partial_obs;
    h->obs_float = cfg->obs_dtype == MRTS_OBS_FLOAT32;
    if (cfg->map_capacity != 0 && cfg->map_capacity < cfg->num_maps)
        return fail(h, MRTS_EINVAL, "map_capacity must be 0 or >= num_maps");
    h->map_capacity = cfg->map_capacity ? cfg->map_capacity : cfg->num_maps;
    h->maps.resize(cfg->num_maps);
    for (int i = 0; i < cfg->num_maps; i++) {
        std::string e;
        if (!cfg->map_paths[i] || !load_map(cfg->map_paths[i], &h->maps[i], &e))
            return fail(h, MRTS_EIO, cfg->map_paths[i] ? e : "null map path");
        h->map_path.emplace_back(cfg->map_paths[i]);
        if (i > 0 && (h->maps[i].w != h->maps[0].w || h->maps[i].h != h->maps[0].h))
            return fail(h, MRTS_EINVAL, "all maps of one vec env must share height x width (vec_env.py:149-150)");
    }
    h->W = h->maps[0].w;
    h->H = h->maps[0].h;
    h->HW = h->W * h->H;
    if (mrts_engine_lds_bytes(h->HW, h->W) > 65536)
        return fail(h, MRTS_ENOTIMPL, "map too large: the step kernel's workgroup LDS carve exceeds 64 KB (maps up to "
                                      "about 1128 cells fit, e.g. 32x32, 33x33, 47x24; DESIGN.md §3)");
    h->game_map.assign(h->ngames, 0);
    for (int g = 0; g < h->ngames; g++) {
        int m = cfg->game_map ? cfg->game_map[g] : 0;
        if (m < 0 || m >= cfg->num_maps) return fail(h, MRTS_EINVAL, "game_map index out of range");
        h->game_map[g] = m;
    }
    h->bot_ai.assign(h->nbot, MRTS_AI_PASSIVE);
    h->nbot_active = 0;
    for (int j = 0; j < h->nbot; j++) {
        int a = cfg->bot_ai ? cfg->bot_ai[j] : MRTS_AI_PASSIVE;
        if (a < 0 || a >= MRTS_AI_COUNT) return fail(h, MRTS_EINVAL, "bot_ai: unknown MRTS_AI_* id");
        h->bot_ai[j] = a;
        h->nbot_active += a != MRTS_AI_PASSIVE;
    }
    if (cfg->game_offset < 0) return fail(h, MRTS_EINVAL, "game_offset must be >= 0");
    h->game_offset = cfg->game_offset;
    h->bot_ai0.assign(h->nbot, -1);
    h->nbot0 = 0;
    for (int j = 0; cfg->bot_ai0 && j < h->nbot; j++) {
        int a = cfg->bot_ai0[j];
        if (a < -1 || a >= MRTS_AI_COUNT) return fail(h, MRTS_EINVAL, "bot_ai0: unknown MRTS_AI_* id");
        h->bot_ai0[j] = a;
        h->nbot0 += a >= 0;
        h->nbot_active += a > MRTS_AI_PASSIVE;
    }
    if (h->nbot_active) {
        if (h->W > 32 || h->H > 64)
            return fail(h, MRTS_ENOTIMPL, "device bots need maps at most 32 wide and 64 high (one bit word per row)");
        if (mrts_engine_bot_lds_bytes(h->HW, h->W) > 65536)
            return fail(h, MRTS_ENOTIMPL, "map too large for the bot kernel's LDS");
    }
    size_t o = 0;
    h->off_cells = o; o = align256(o + (size_t)h->ngames * cell_stride(h->HW) * sizeof(int4));
    h->off_genv = o; o = align256(o + (size_t)h->ngames * MRTS_GENV_WORDS * sizeof(int32_t));
    h->off_mcells = o; o = align256(o + (size_t)h->map_capacity * h->HW * sizeof(int4));
    h->off_mwall = o; o = align256(o + (size_t)h->map_capacity * h->HW);
    h->off_mscal = o; o = align256(o + (size_t)h->map_capacity * MRTS_MAP_SCALARS * sizeof(int32_t));
    h->off_scratch = o; o = align256(o + (size_t)2 * h->ngames * sizeof(int32_t));
    h->off_botai = o; o = align256(o + (size_t)(h->nbot + 1) * sizeof(int32_t));
    h->off_botai0 = o; o = align256(o + (size_t)(h->nbot + 1) * sizeof(int32_t));
    h->off_aa = o; o = align256(o + (h->nbot_active ? (size_t)h->nbot * 2 * h->HW * 2 * sizeof(int4) : 0));
    h->off_botpa = o; o = align256(o + (h->nbot_active ? (size_t)h->nbot * 2 * h->HW * sizeof(int32_t) : 0));
    h->off_parked = o; o = align256(o + (size_t)h->ngames);
    h->total = o;
    h->err.clear();
    return MRTS_OK;
}

int mrts_info(const mrts_vec *h, mrts_info_t *info) {
    if (!h || !info || h->HW == 0) return MRTS_EINVAL;
    info->height = h->H;
    info->width = h->W;
    info->num_envs = h->nenvs;
    info->num_games = h->ngames;
    info->obs_planes = h->partial_obs ? 31 : 29;
    info->mask_channels = MRTS_MASK_CH;
    info->action_components = 7;
    info->workspace_bytes = h->total;
    return MRTS_OK;
}

int mrts_bind_workspace(mrts_vec *h, void *dev, void *stream) {
    if (!h || !dev || h->HW == 0) return fail(h, MRTS_EINVAL, "bind_workspace: bad handle or pointer");
    if (((uintptr_t)dev & 255u) != 0) return fail(h, MRTS_EINVAL, "workspace must be 256-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    h->bots_ready = false;
    h->ws = (unsigned char *)dev;
    const int nm = (int)h->maps.size();
    std::vector<int4> mc((size_t)nm * h->HW);
    std::vector<uint8_t> mw((size_t)nm * h->HW);
    std::vector<int32_t> ms((size_t)nm * MRTS_MAP_SCALARS, 0);
    for (int i = 0; i < nm; i++) {
        std::memcpy(&mc[(size_t)i * h->HW], h->maps[i].cells.data(), sizeof(int4) * h->HW);
        std::memcpy(&mw[(size_t)i * h->HW], h->maps[i].wall.data(), h->HW);
        ms[i * MRTS_MAP_SCALARS + MRTS_M_RES0] = h->maps[i].res[0];
        ms[i * MRTS_MAP_SCALARS + MRTS_M_RES1] = h->maps[i].res[1];
        ms[i * MRTS_MAP_SCALARS + MRTS_M_NUNITS] = h->maps[i].nunits;
    }
    std::vector<int32_t> genv((size_t)h->ngames * MRTS_GENV_WORDS, 0);
    for (int g = 0; g < h->ngames; g++) genv[(size_t)g * MRTS_GENV_WORDS + MRTS_G_MAP] = h->game_map[g];
    hipError_t e;
    if ((e = hipMemcpyAsync(h->ws + h->off_mcells, mc.data(), mc.size() * sizeof(int4), hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(h->ws + h->off_mwall, mw.data(), mw.size(), hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(h->ws + h->off_mscal, ms.data(), ms.size() * sizeof(int32_t), hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(h->ws + h->off_genv, genv.data(), genv.size() * sizeof(int32_t), hipMemcpyHostToDevice, s)) ||
        (h->nbot && (e = hipMemcpyAsync(h->ws + h->off_botai, h->bot_ai.data(), h->nbot * sizeof(int32_t), hipMemcpyHostToDevice, s))) ||
        (h->nbot && (e = hipMemcpyAsync(h->ws + h->off_botai0, h->bot_ai0.data(), h->nbot * sizeof(int32_t), hipMemcpyHostToDevice, s))) ||
        (e = hipStreamSynchronize(s)))
        return hip_fail(h, e, "bind_workspace upload");
    EngineParams &p = h->base;
    p = EngineParams{};
    p.cells = (int4 *)(h->ws + h->off_cells);
    p.cstride = cell_stride(h->HW);
    p.genv = (int32_t *)(h->ws + h->off_genv);
    p.map_cells = (const int4 *)(h->ws + h->off_mcells);
    p.map_wall = (const uint8_t *)(h->ws + h->off_mwall);
    p.map_scal = (const int32_t *)(h->ws + h->off_mscal);
    p.G = h->ngames;
    p.nmaps = (int)h->maps.size();
    p.HW = h->HW;
    p.W = h->W;
    p.H = h->H;
    p.nsp = h->nsp;
    p.nsp_games = h->nsp / 2;
    p.max_steps = h->max_steps;
    p.obs_float = h->obs_float;
    p.partial_obs = h->partial_obs;
    p.bot_ai = (const int32_t *)(h->ws + h->off_botai);
    p.bot_ai0 = h->nbot0 ? (const int32_t *)(h->ws + h->off_botai0) : nullptr;
    p.aa = h->nbot_active ? (int4 *)(h->ws + h->off_aa) : nullptr;
    p.botpa = h->nbot_active ? (int32_t *)(h->ws + h->off_botpa) : nullptr;
    p.nbot_active = h->nbot_active;
    p.game_offset = h->game_offset;
    p.early_bot = mrts_engine_early_bot_ok(h->HW, h->W);
    p.parked = nullptr;   // until a game is parked
    h->parked.assign(h->ngames, 0);
    h->err.clear();
    return MRTS_OK;
}

// host flags -> device; the engine checks them from now on
static hipError_t upload_parked(mrts_vec *h, hipStream_t s) {
    uint8_t *d = h->ws + h->off_parked;
    hipError_t e = hipMemcpyAsync(d, h->parked.data(), h->parked.size(), hipMemcpyHostToDevice, s);
    if (!e) e = hipStreamSynchronize(s);   // the host vector may change before the copy would run
    if (!e) h->base.parked = d;
    return e;
}

static bool bound(mrts_vec *h) { return h && h->ws; }

// Bot fusion applies to games whose bots play player 1 only (bot-vs-bot games
// decide for both sides: separate k_bot), and when both LDS regions fit a
// workgroup (the fused step workgroup has at least two waves: maps of <= 64
// cells take 128 lanes, mrts_engine.hip step_nt).
static bool fused(const mrts_vec *h) {
    return h->fuse && h->nbot_active > 0 && h->nbot0 == 0 && mrts_engine_fused_lds_bytes(h->HW, h->W, h->partial_obs) <= 163840;
}

// k_bot (when the tick's bot decisions are not already there) + k_step on s
static hipError_t step_launch(mrts_vec *h, EngineParams &p, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (!h->bots_ready) e = mrts_engine_bots(&p, s);
    p.fuse_bots = fused(h) ? 1 : 0;
    if (!e) e = mrts_engine_step(&p, s);
    h->bots_ready = p.fuse_bots != 0;
    return e;
}

// after a reset of every game (games == null) or of the listed ones: with
// fusion, decide their bot actions now (the next step will not launch k_bot)
static hipError_t bots_after_reset(mrts_vec *h, hipStream_t s, const int32_t *games, int count) {
    if (!fused(h)) {
        h->bots_ready = false;
        return hipSuccess;
    }
    if (games && !h->bots_ready) return hipSuccess;   // the next step decides for every game anyway
    EngineParams p = h->base;
    p.bot_games = games;
    p.bot_ngames = count;
    hipError_t e = mrts_engine_bots(&p, s);
    if (!e) h->bots_ready = true;
    return e;
}

int mrts_set_bot_fusion(mrts_vec *h, int32_t on) {
    if (!h) return fail(h, MRTS_EINVAL, "set_bot_fusion: null handle");
    h->fuse = on ? 1 : 0;   // bots_ready stays valid: decisions already made are used once either way
    return MRTS_OK;
}

int mrts_reset(mrts_vec *h, void *stream, void *obs) {
    if (!bound(h) || !obs) return fail(h, MRTS_ESTATE, "reset: workspace not bound or obs null");
    EngineParams p = h->base;
    p.obs = obs;
    p.mask = h->next_mask;
    p.src_out = h->next_src;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = mrts_engine_reset(&p, s, nullptr, nullptr, 0);
    if (!e) e = bots_after_reset(h, s, nullptr, 0);
    return e ? hip_fail(h, e, "reset launch") : MRTS_OK;
}

int mrts_get_masks(mrts_vec *h, void *stream, int32_t *mask, int32_t *source) {
    if (!bound(h) || !mask || !source) return fail(h, MRTS_ESTATE, "get_masks: workspace not bound or null output");
    EngineParams p = h->base;
    p.mask = mask;
    p.src_out = source;
    hipError_t e = mrts_engine_masks(&p, (hipStream_t)stream);
    return e ? hip_fail(h, e, "masks launch") : MRTS_OK;
}

// the step's parameters of one engine (mrts_step / mrts_step_weighted / mrts_step_group)
static EngineParams step_params(const mrts_vec *h, const mrts_step_io &io) {
    EngineParams p = h->base;
    p.actions = io.actions;
    p.src = io.source;
    p.obs = io.obs;
    p.raw_reward = io.raw_reward;
    p.done = io.done;
    if (io.reward) {
        p.reward = io.reward;
        p.done0 = io.done0;
        for (int k = 0; k < 6; k++) p.rw[k] = h->rw[k];
        p.shaping = h->shaping;
    }
    p.mask = h->next_mask;
    p.src_out = h->next_src;
    return p;
}

static bool io_ok(const mrts_step_io &io, bool weighted) {
    return io.actions && io.source && io.obs && io.raw_reward && io.done && (!weighted || (io.reward && io.done0));
}

int mrts_step(mrts_vec *h, void *stream, const int64_t *actions, const int32_t *source, void *obs, double *raw_reward,
              uint8_t *done) {
    const mrts_step_io io{actions, source, obs, raw_reward, done, nullptr, nullptr};
    if (!bound(h) || !io_ok(io, false)) return fail(h, MRTS_ESTATE, "step: workspace not bound or null buffer");
    EngineParams p = step_params(h, io);
    hipError_t e = step_launch(h, p, (hipStream_t)stream);
    return e ? hip_fail(h, e, "step launch") : MRTS_OK;
}

int mrts_get_raw_obs(mrts_vec *h, void *stream, int32_t *raw) {
    if (!bound(h) || !raw) return fail(h, MRTS_ESTATE, "get_raw_obs: workspace not bound or raw null");
    hipError_t e = mrts_engine_raw_obs(&h->base, (hipStream_t)stream, raw);
    return e ? hip_fail(h, e, "raw obs launch") : MRTS_OK;
}

int mrts_set_reward_weight(mrts_vec *h, const double *w, int32_t shaping) {
    if (!h || !w) return fail(h, MRTS_EINVAL, "set_reward_weight: null argument");
    for (int k = 0; k < 6; k++) h->rw[k] = w[k];
    h->shaping = shaping ? 1 : 0;
    return MRTS_OK;
}

int mrts_step_weighted(mrts_vec *h, void *stream, const int64_t *actions, const int32_t *source, void *obs,
                       double *raw_reward, uint8_t *done, double *reward, uint8_t *done0) {
    const mrts_step_io io{actions, source, obs, raw_reward, done, reward, done0};
    if (!bound(h) || !io_ok(io, true)) return fail(h, MRTS_ESTATE, "step_weighted: workspace not bound or null buffer");
    EngineParams p = step_params(h, io);
    hipError_t e = step_launch(h, p, (hipStream_t)stream);
    return e ? hip_fail(h, e, "step launch") : MRTS_OK;
}

// A member may share a launch when its workgroup still leaves >= this many per CU
// at the widest workgroup size: the step kernels' own occupancy (6-7 workgroups
// per CU, register-limited), so that merging costs no member residency; a larger
// map keeps its own launch.  (configs[4], round 4: 24x24 apart at 40 KB 261 us per
// step vs 264 us all in one launch, profiles/r04_ab/.)
#ifndef MRTS_GROUP_MIN_WG_PER_CU
#define MRTS_GROUP_MIN_WG_PER_CU 6
#endif
static const size_t kGroupLdsCap = 163840 / MRTS_GROUP_MIN_WG_PER_CU;

// Launch plan of a group: launch_of[i] = the launch (0, 1, ..) member i runs in.
// Members of equal planes / obs type / fusion share a launch (merge != 0), each
// launch in the caller's order of its first member.  Returns the launch count.
static int group_plan(const EngineParams *ps, int n, int policy, int *launch_of) {
    const int merge = policy & 3;
    auto lds = [&](const EngineParams &p, int NT) { return mrts_engine_group_lds_bytes(p.HW, p.W, p.fuse_bots, NT, p.partial_obs); };
    auto compatible = [&](const EngineParams &a, const EngineParams &b) {
        return a.partial_obs == b.partial_obs && a.obs_float == b.obs_float && (a.fuse_bots != 0) == (b.fuse_bots != 0);
    };
    for (int i = 0; i < n; i++) launch_of[i] = -1;
    int nl = 0;
    for (int i = 0; i < n; i++) {
        if (launch_of[i] >= 0) continue;
        int NT = mrts_engine_step_nt(ps[i].HW, ps[i].fuse_bots);
        launch_of[i] = nl;
        for (int j = i + 1; merge && j < n; j++) {
            if (launch_of[j] >= 0 || !compatible(ps[i], ps[j])) continue;
            const int NT2 = std::max(NT, mrts_engine_step_nt(ps[j].HW, ps[j].fuse_bots));
            bool fits = true;
            if (merge == MRTS_GROUP_MERGE_FIT)
                for (int k = 0; k < n; k++)
                    if ((k == j || launch_of[k] == nl) && lds(ps[k], NT2) > kGroupLdsCap) fits = false;
            if (!fits) continue;
            launch_of[j] = nl;
            NT = NT2;
        }
        nl++;
    }
    return nl;
}

// A group call's error is recorded on the member it concerns AND on hs[0], the
// handle callers read mrts_last_error from (a failure of member i > 0
// used to leave hs[0]'s message empty or stale).
static int group_fail(mrts_vec *const *hs, int i, int code, const std::string &msg) {
    const std::string m = i > 0 ? msg + " (member " + std::to_string(i) + ")" : msg;
    if (hs && i >= 0 && hs[i]) hs[i]->err = m;
    if (hs && hs[0]) hs[0]->err = m;
    return code;
}

static int group_check(mrts_vec *const *hs, int32_t n, const mrts_step_io *io, int32_t policy, bool need_bound = true) {
    if (!hs || n < 1 || n > MRTS_STEP_GROUP_MAX) return fail(hs && n >= 1 ? hs[0] : nullptr, MRTS_EINVAL, "step_group: bad arguments");
    if ((policy & ~7) || (policy & 3) == 3) return group_fail(hs, 0, MRTS_EINVAL, "step_group: unknown policy bits");
    for (int i = 0; i < n; i++) {
        if (!hs[i]) return group_fail(hs, i, MRTS_EINVAL, "step_group: null handle");
        if ((need_bound && !bound(hs[i])) || (io && !io_ok(io[i], io[i].reward != nullptr)))
            return group_fail(hs, i, MRTS_ESTATE, "step_group: workspace not bound or null buffer");
        for (int j = 0; j < i; j++)
            if (hs[j] == hs[i]) return group_fail(hs, i, MRTS_EINVAL, "step_group: an engine listed twice");
    }
    return MRTS_OK;
}

int mrts_step_group_plan(mrts_vec *const *hs, int32_t n, int32_t policy, int32_t *launch_of, int32_t *launches) {
    int rc = group_check(hs, n, nullptr, policy, false);   // a plan needs only the handles' configs
    if (rc) return rc;
    if (!launch_of || !launches) return fail(hs[0], MRTS_EINVAL, "step_group_plan: null output");
    EngineParams ps[MRTS_STEP_GROUP_MAX];
    int lo[MRTS_STEP_GROUP_MAX];
    for (int i = 0; i < n; i++) {
        ps[i] = EngineParams{};
        ps[i].HW = hs[i]->HW;
        ps[i].W = hs[i]->W;
        ps[i].partial_obs = hs[i]->partial_obs;
        ps[i].obs_float = hs[i]->obs_float;
        ps[i].fuse_bots = fused(hs[i]) ? 1 : 0;
    }
    *launches = group_plan(ps, n, policy, lo);
    for (int i = 0; i < n; i++) launch_of[i] = lo[i];
    return MRTS_OK;
}

int mrts_step_group(mrts_vec *const *hs, int32_t n, void *stream, const mrts_step_io *io, int32_t policy) {
    int rc = group_check(hs, n, io, policy);
    if (rc) return rc;
    if (!io) return group_fail(hs, 0, MRTS_EINVAL, "step_group: null io");
    hipStream_t s = (hipStream_t)stream;
    EngineParams ps[MRTS_STEP_GROUP_MAX];
    for (int i = 0; i < n; i++) {
        mrts_vec *h = hs[i];
        ps[i] = step_params(h, io[i]);
        // the tick's bot decisions, when an earlier launch did not make them
        hipError_t e = h->bots_ready ? hipSuccess : mrts_engine_bots(&ps[i], s);
        if (e) return group_fail(hs, i, MRTS_EHIP, std::string("step_group bot launch: ") + hipGetErrorString(e));
        h->bots_ready = true;   // this tick's decisions are in botpa now, whatever happens below
        ps[i].fuse_bots = fused(h) ? 1 : 0;
    }
    int launch_of[MRTS_STEP_GROUP_MAX];
    const int nl = group_plan(ps, n, policy, launch_of);
    for (int l = 0; l < nl; l++) {
        EngineParams grp[MRTS_STEP_GROUP_MAX];
        int m = 0, first = -1;
        for (int i = 0; i < n; i++)
            if (launch_of[i] == l) {
                if (first < 0) first = i;
                grp[m++] = ps[i];
            }
        hipError_t e = mrts_engine_step_group(grp, m, s, (policy & MRTS_GROUP_BOTS_FIRST) != 0);
        // not atomic: members of launches 0..l-1 have stepped, those of l.. have not
        // (include/microrts_amd.h); each member's bot state follows its own launch
        if (e) return group_fail(hs, first, MRTS_EHIP, std::string("step_group launch: ") + hipGetErrorString(e));
        for (int i = 0; i < n; i++)
            if (launch_of[i] == l) hs[i]->bots_ready = ps[i].fuse_bots != 0;
    }
    return MRTS_OK;
}

int mrts_reset_games(mrts_vec *h, void *stream, const int32_t *games, const int32_t *maps, int32_t count, void *obs) {
    if (!bound(h) || !obs || count < 0 || count > h->ngames || (count && (!games || !maps)))
        return fail(h, MRTS_EINVAL, "reset_games: bad arguments");
    if (count == 0) return MRTS_OK;
    for (int i = 0; i < count; i++) {
        if (games[i] < 0 || games[i] >= h->ngames || maps[i] < 0 || maps[i] >= (int)h->maps.size())
            return fail(h, MRTS_EINVAL, "reset_games: index out of range");
        h->game_map[games[i]] = maps[i];
    }
    hipStream_t s = (hipStream_t)stream;
    if (h->base.parked) {   // the listed games play again
        bool any = false;
        for (int i = 0; i < count; i++) {
            any |= h->parked[games[i]] != 0;
            h->parked[games[i]] = 0;
        }
        if (any) {
            hipError_t e = upload_parked(h, s);
            if (e) return hip_fail(h, e, "reset_games unpark");
        }
    }
    h->scratch_host.assign(games, games + count);
    h->scratch_host.insert(h->scratch_host.end(), maps, maps + count);
    int32_t *dg = (int32_t *)(h->ws + h->off_scratch);
    hipError_t e = hipMemcpyAsync(dg, h->scratch_host.data(), sizeof(int32_t) * 2 * count, hipMemcpyHostToDevice, s);
    if (e) return hip_fail(h, e, "reset_games upload");
    EngineParams p = h->base;
    p.obs = obs;
    p.mask = h->next_mask;
    p.src_out = h->next_src;
    e = mrts_engine_reset(&p, s, dg, dg + count, count);
    if (!e) e = bots_after_reset(h, s, dg, count);
    if (e) return hip_fail(h, e, "reset_games launch");
    // the host staging vector must outlive the copy
    e = hipStreamSynchronize(s);
    return e ? hip_fail(h, e, "reset_games sync") : MRTS_OK;
}

int mrts_add_map(mrts_vec *h, void *stream, const char *path, int32_t *index) {
    if (!bound(h) || !path || !index) return fail(h, MRTS_EINVAL, "add_map: not bound or null argument");
    for (size_t i = 0; i < h->map_path.size(); i++)
        if (h->map_path[i] == path) {
            *index = (int32_t)i;
            return MRTS_OK;
        }
    if ((int)h->maps.size() >= h->map_capacity) return fail(h, MRTS_EINVAL, "add_map: every map slot is taken (map_capacity)");
    MapData m;
    std::string err;
    if (!load_map(path, &m, &err)) return fail(h, MRTS_EIO, err);
    if (m.w != h->W || m.h != h->H)
        return fail(h, MRTS_EINVAL, "add_map: all maps of one vec env must share height x width (vec_env.py:149-150)");
    const int i = (int)h->maps.size();
    int32_t scal[MRTS_MAP_SCALARS] = {0};
    scal[MRTS_M_RES0] = m.res[0];
    scal[MRTS_M_RES1] = m.res[1];
    scal[MRTS_M_NUNITS] = m.nunits;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    // a slot no game uses yet: nothing in flight reads it
    if ((e = hipMemcpyAsync(h->ws + h->off_mcells + (size_t)i * h->HW * sizeof(int4), m.cells.data(), sizeof(int4) * h->HW,
                            hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(h->ws + h->off_mwall + (size_t)i * h->HW, m.wall.data(), h->HW, hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(h->ws + h->off_mscal + (size_t)i * MRTS_MAP_SCALARS * sizeof(int32_t), scal, sizeof(scal),
                            hipMemcpyHostToDevice, s)) ||
        (e = hipStreamSynchronize(s)))
        return hip_fail(h, e, "add_map upload");
    h->maps.push_back(std::move(m));
    h->map_path.emplace_back(path);
    h->base.nmaps = (int)h->maps.size();
    *index = i;
    return MRTS_OK;
}

int mrts_park_games(mrts_vec *h, void *stream, const int32_t *games, int32_t count, void *obs) {
    if (!bound(h) || !obs || count < 0 || count > h->ngames || (count && !games))
        return fail(h, MRTS_EINVAL, "park_games: bad arguments");
    if (count == 0) return MRTS_OK;
    for (int i = 0; i < count; i++) {
        if (games[i] < 0 || games[i] >= h->ngames) return fail(h, MRTS_EINVAL, "park_games: game out of range");
        h->parked[games[i]] = 1;
    }
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = upload_parked(h, s);
    if (e) return hip_fail(h, e, "park_games upload");
    // k_reset over the list: parked games write zero obs / masks / sources
    h->scratch_host.assign(games, games + count);
    h->scratch_host.insert(h->scratch_host.end(), games, games + count);   // (map list unused for parked games)
    int32_t *dg = (int32_t *)(h->ws + h->off_scratch);
    if ((e = hipMemcpyAsync(dg, h->scratch_host.data(), sizeof(int32_t) * 2 * count, hipMemcpyHostToDevice, s)))
        return hip_fail(h, e, "park_games upload");
    EngineParams p = h->base;
    p.obs = obs;
    p.mask = h->next_mask;
    p.src_out = h->next_src;
    e = mrts_engine_reset(&p, s, dg, dg + count, count);
    if (!e) e = hipStreamSynchronize(s);
    return e ? hip_fail(h, e, "park_games launch") : MRTS_OK;
}

int mrts_sample_actions(void *stream, const int32_t *mask, int32_t n, int32_t hw, int32_t env0, uint64_t seed, uint32_t step,
                        int64_t *actions) {
    if (!mask || !actions || n < 0 || hw <= 0 || env0 < 0) return MRTS_EINVAL;
    return mrts_engine_sample(mask, n, hw, env0, seed, step, actions, (hipStream_t)stream) ? MRTS_EHIP : MRTS_OK;
}

int mrts_sample_actions_src(void *stream, const int32_t *mask, const int32_t *source, int32_t n, int32_t hw, int32_t env0,
                            uint64_t seed, uint32_t step, int64_t *actions) {
    if (!mask || !source || !actions || n < 0 || hw <= 0 || env0 < 0) return MRTS_EINVAL;
    if ((int64_t)n * hw > (int64_t)INT32_MAX - 256) return MRTS_EINVAL;   // k_sample_src indexes rows in 32 bits
    return mrts_engine_sample_src(mask, source, n, hw, env0, seed, step, actions, (hipStream_t)stream) ? MRTS_EHIP : MRTS_OK;
}

int mrts_sample_actions_src_group(void *stream, const mrts_sample_seg *segs, int32_t nseg, uint64_t seed, uint32_t step) {
    if (!segs || nseg < 1 || nseg > MRTS_SAMPLE_GROUP_MAX) return MRTS_EINVAL;
    for (int k = 0; k < nseg; k++) {
        const mrts_sample_seg &q = segs[k];
        if (!q.mask || !q.source || !q.actions || q.num_envs < 0 || q.hw <= 0 || q.env0 < 0) return MRTS_EINVAL;
        if ((int64_t)q.num_envs * q.hw > (int64_t)INT32_MAX - 256) return MRTS_EINVAL;   // 32-bit row indexing
        if ((uintptr_t)q.actions & 15u) return MRTS_EINVAL;   // the rows' 16-byte stores
    }
    return mrts_engine_sample_src_group(segs, nseg, seed, step, (hipStream_t)stream) ? MRTS_EHIP : MRTS_OK;
}

int mrts_bind_mask_outputs(mrts_vec *h, int32_t *mask, int32_t *source) {
    if (!bound(h)) return fail(h, MRTS_ESTATE, "bind_mask_outputs: workspace not bound");
    if ((mask == nullptr) != (source == nullptr)) return fail(h, MRTS_EINVAL, "bind_mask_outputs: mask and source go together");
    if (mask && ((uintptr_t)mask & 15u)) return fail(h, MRTS_EINVAL, "bind_mask_outputs: mask must be 16-byte aligned");
    h->next_mask = mask;
    h->next_src = source;
    return MRTS_OK;
}

int mrts_render(mrts_vec *h, void *stream, int32_t env, uint8_t *rgb, int32_t size) {
    if (!bound(h) || !rgb) return fail(h, MRTS_ESTATE, "render: workspace not bound or rgb null");
    if (env < 0 || env >= h->nenvs) return fail(h, MRTS_EINVAL, "render: env out of range");
    if (size < h->W || size < h->H || size > 8192) return fail(h, MRTS_EINVAL, "render: size must be in [max(H, W), 8192]");
    const int game = env < h->nsp ? env / 2 : h->nsp / 2 + (env - h->nsp);
    hipError_t e = mrts_engine_render(&h->base, (hipStream_t)stream, game, h->game_map[game], size, rgb);
    return e ? hip_fail(h, e, "render launch") : MRTS_OK;
}

// Env-state checkpoint: [header | workspace bytes].  The header carries what the
// host holds beside the workspace (bots_ready, the games' map indices, parked flags),
// the shape the snapshot belongs to and a fingerprint of the configuration whose
// device tables the workspace copy brings along (bots, map templates): a snapshot
// loads only into a handle of the same shape AND configuration.
namespace {
struct StateHeader {
    uint32_t magic, version;
    int32_t ngames, HW, nmaps, bots_ready, parked_any;
    uint64_t total;
    uint64_t config;   // config_fingerprint
};
const uint32_t kStateMagic = 0x4d525453u;   // "MRTS"
const uint32_t kStateVersion = 3;
size_t state_header_bytes(const mrts_vec *h) {
    return align256(sizeof(StateHeader) + (size_t)h->ngames * (sizeof(int32_t) + 1));
}
struct Fnv {
    uint64_t v = 1469598103934665603ull;
    void bytes(const void *p, size_t n) {
        const unsigned char *b = (const unsigned char *)p;
        for (size_t i = 0; i < n; i++) v = (v ^ b[i]) * 1099511628211ull;
    }
    void i32(int32_t x) { bytes(&x, sizeof x); }
};
// FNV-1a over everything a workspace copy would carry in besides the game states:
// env split, obs layout, global game offset (bot RNG streams), the time limit, the
// bots of every bot env (both players), the map table's capacity and every map
// template (size, resources, walls, unit records).  Not the reward weights / shaping:
// the caller may reassign those between steps (vec_env.py reads reward_weight every step).
uint64_t config_fingerprint(const mrts_vec *h) {
    Fnv f;
    for (int32_t x : {h->nsp, h->nbot, h->partial_obs, h->obs_float, h->game_offset, h->map_capacity, h->W, h->H,
                      h->max_steps})
        f.i32(x);
    f.i32((int32_t)h->bot_ai.size());
    f.bytes(h->bot_ai.data(), h->bot_ai.size() * sizeof(int32_t));
    f.i32((int32_t)h->bot_ai0.size());
    f.bytes(h->bot_ai0.data(), h->bot_ai0.size() * sizeof(int32_t));
    f.i32((int32_t)h->maps.size());
    for (const MapData &m : h->maps) {
        for (int32_t x : {m.w, m.h, m.res[0], m.res[1], m.nunits}) f.i32(x);
        f.bytes(m.wall.data(), m.wall.size());
        f.bytes(m.cells.data(), m.cells.size() * sizeof(int4));
    }
    return f.v;
}
}  // namespace

size_t mrts_state_bytes(const mrts_vec *h) { return bound(const_cast<mrts_vec *>(h)) ? state_header_bytes(h) + h->total : 0; }

int mrts_save_state(mrts_vec *h, void *stream, void *dst) {
    if (!bound(h) || !dst) return fail(h, MRTS_ESTATE, "save_state: workspace not bound or dst null");
    if (((uintptr_t)dst & 255u) != 0) return fail(h, MRTS_EINVAL, "save_state: dst must be 256-byte aligned");
    std::vector<unsigned char> hdr(state_header_bytes(h), 0);
    StateHeader sh{kStateMagic, kStateVersion, h->ngames, h->HW, (int32_t)h->maps.size(), h->bots_ready ? 1 : 0,
                   h->base.parked != nullptr ? 1 : 0, (uint64_t)h->total, config_fingerprint(h)};
    std::memcpy(hdr.data(), &sh, sizeof sh);
    std::memcpy(hdr.data() + sizeof sh, h->game_map.data(), (size_t)h->ngames * sizeof(int32_t));
    std::memcpy(hdr.data() + sizeof sh + (size_t)h->ngames * sizeof(int32_t), h->parked.data(), (size_t)h->ngames);
    hipStream_t s = (hipStream_t)stream;
    unsigned char *d = (unsigned char *)dst;
    hipError_t e = hipMemcpyAsync(d, hdr.data(), hdr.size(), hipMemcpyHostToDevice, s);
    if (!e) e = hipMemcpyAsync(d + hdr.size(), h->ws, h->total, hipMemcpyDeviceToDevice, s);
    // the host header buffer is this call's: drain the stream on every path (a queued
    // copy may still read it after a later enqueue failed)
    const hipError_t es = hipStreamSynchronize(s);
    if (!e) e = es;
    return e ? hip_fail(h, e, "save_state copy") : MRTS_OK;
}

int mrts_load_state(mrts_vec *h, void *stream, const void *src, void *obs) {
    if (!bound(h) || !src || !obs) return fail(h, MRTS_ESTATE, "load_state: workspace not bound or null buffer");
    if (((uintptr_t)src & 255u) != 0) return fail(h, MRTS_EINVAL, "load_state: src must be 256-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    // the fixed header first: a snapshot of a smaller handle is shorter than this
    // handle's header, so nothing beyond sizeof(StateHeader) is read before it checks out
    StateHeader sh;
    hipError_t e = hipMemcpyAsync(&sh, src, sizeof sh, hipMemcpyDeviceToHost, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return hip_fail(h, e, "load_state header");
    if (sh.magic != kStateMagic || sh.version != kStateVersion)
        return fail(h, MRTS_EINVAL, "load_state: not a snapshot of this library version (mrts_save_state)");
    if (sh.ngames != h->ngames || sh.HW != h->HW || sh.nmaps != (int32_t)h->maps.size() || sh.total != (uint64_t)h->total)
        return fail(h, MRTS_EINVAL, "load_state: the snapshot belongs to another configuration or map table");
    if (sh.config != config_fingerprint(h))
        return fail(h, MRTS_EINVAL, "load_state: the snapshot belongs to another configuration (bots, maps, obs layout, "
                                    "game offset or max_steps differ)");
    std::vector<unsigned char> hdr(state_header_bytes(h), 0);
    e = hipMemcpyAsync(hdr.data(), src, hdr.size(), hipMemcpyDeviceToHost, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return hip_fail(h, e, "load_state header");
    e = hipMemcpyAsync(h->ws, (const unsigned char *)src + hdr.size(), h->total, hipMemcpyDeviceToDevice, s);
    if (e) return hip_fail(h, e, "load_state copy");
    // the host mirrors only once the workspace copy is queued: a failed copy leaves them as they were
    std::memcpy(h->game_map.data(), hdr.data() + sizeof sh, (size_t)h->ngames * sizeof(int32_t));
    std::memcpy(h->parked.data(), hdr.data() + sizeof sh + (size_t)h->ngames * sizeof(int32_t), (size_t)h->ngames);
    h->bots_ready = sh.bots_ready != 0;
    h->base.parked = sh.parked_any ? (uint8_t *)(h->ws + h->off_parked) : nullptr;
    EngineParams p = h->base;
    p.obs = obs;
    p.mask = h->next_mask;
    p.src_out = h->next_src;
    e = mrts_engine_outputs(&p, s);
    return e ? hip_fail(h, e, "load_state outputs launch") : MRTS_OK;
}

int mrts_game_stats(mrts_vec *h, void *stream, int32_t *out) {
    if (!bound(h) || !out) return fail(h, MRTS_ESTATE, "game_stats: not bound or out null");
    std::vector<int32_t> genv((size_t)h->ngames * MRTS_GENV_WORDS);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(genv.data(), h->ws + h->off_genv, genv.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return hip_fail(h, e, "game_stats readback");
    static const int words[MRTS_GAME_STATS] = {MRTS_G_TIME, MRTS_G_STEPS, MRTS_G_TICKS, MRTS_G_SERIAL, MRTS_G_ORDERED, MRTS_G_EPISODES};
    for (int g = 0; g < h->ngames; g++)
        for (int k = 0; k < MRTS_GAME_STATS; k++) out[(size_t)g * MRTS_GAME_STATS + k] = genv[(size_t)g * MRTS_GENV_WORDS + words[k]];
    return MRTS_OK;
}

int mrts_error_flags(mrts_vec *h, void *stream, int32_t *flags_out) {
    if (!bound(h) || !flags_out) return fail(h, MRTS_ESTATE, "error_flags: not bound");
    std::vector<int32_t> genv((size_t)h->ngames * MRTS_GENV_WORDS);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(genv.data(), h->ws + h->off_genv, genv.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return hip_fail(h, e, "error_flags readback");
    int32_t f = 0;
    for (int g = 0; g < h->ngames; g++) f |= genv[(size_t)g * MRTS_GENV_WORDS + MRTS_G_ERR];
    *flags_out = f;
    return MRTS_OK;
}

int mrts_fused_layout_ok(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0 || width > 32 || height > 64) return -1;
    const int HW = width * height;
    if (mrts_engine_fused_lds_bytes(HW, width, 0) > 163840) return -1;
    if (mrts_engine_bot_lds_bytes(HW, width) > 65536) return -1;   // mrts_create refuses such bot engines
    return mrts_engine_early_bot_ok(HW, width);
}

const char *mrts_utt_json(const mrts_vec *h) { return h ? h->utt.c_str() : ""; }
const char *mrts_last_error(const mrts_vec *h) { return h ? h->err.c_str() : "null handle"; }
void mrts_destroy(mrts_vec *h) { delete h; }

}  // extern "C"
