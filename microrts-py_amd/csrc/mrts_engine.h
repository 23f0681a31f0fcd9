// mrts_engine.h -- internal launch interface between the C ABI (mrts_capi.cpp)
// and the kernels (mrts_engine.hip).
#ifndef MRTS_ENGINE_H
#define MRTS_ENGINE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "microrts_amd.h"   // mrts_sample_seg, MRTS_* limits

// Phase stamps (tracing, experiment builds only: `make STAMPS=1`): each step
// workgroup takes a row of g_stamp and writes wall_clock64() (100 MHz) at its
// phase boundaries; mrts_debug_stamps (mrts_engine.hip) reads the rows back.
// Compiled out of the product library.
#ifdef MRTS_STAMPS
#define MRTS_STAMP_ROWS 65536
#define MRTS_STAMP_COLS 20   // 2..15 phase stamps, 16..19 bot counters (MRTS_STAMP_ADD)
static __device__ unsigned long long g_stamp[MRTS_STAMP_ROWS][MRTS_STAMP_COLS];
__shared__ int mrts_stamp_row;
// mrts_stamp_row: set by k_step's thread 0 before a barrier; every other kernel
// that reaches a stamp site (k_reset / k_masks through emit_outputs) sets it to -1
// first (MRTS_STAMP_NONE), and the unsigned bound check skips it
#define MRTS_STAMP(k, cond) \
    do { if ((cond) && (unsigned)mrts_stamp_row < (unsigned)MRTS_STAMP_ROWS) g_stamp[mrts_stamp_row][k] = wall_clock64(); } while (0)
#define MRTS_STAMP_MAX(k, cond) \
    do { if ((cond) && (unsigned)mrts_stamp_row < (unsigned)MRTS_STAMP_ROWS) \
             atomicMax(&g_stamp[mrts_stamp_row][k], (unsigned long long)wall_clock64()); } while (0)
#define MRTS_STAMP_NONE() do { if (threadIdx.x == 0) mrts_stamp_row = -1; __syncthreads(); } while (0)
// a counter of the row (one writer: the bot wave's lane 0)
#define MRTS_STAMP_ADD(k, v, cond) \
    do { if ((cond) && (unsigned)mrts_stamp_row < (unsigned)MRTS_STAMP_ROWS) g_stamp[mrts_stamp_row][k] += (v); } while (0)
#else
#define MRTS_STAMP(k, cond) do { } while (0)
#define MRTS_STAMP_MAX(k, cond) do { } while (0)
#define MRTS_STAMP_NONE() do { } while (0)
#define MRTS_STAMP_ADD(k, v, cond) do { } while (0)
#endif

struct EngineParams {
    int4 *cells;            // [G][cstride] (the first HW records of each game's row)
    int cstride;            // int4 records between consecutive games' cells (>= HW)
    int32_t *genv;          // [G][MRTS_GENV_WORDS]
    const int4 *map_cells;  // [maps][HW]
    const uint8_t *map_wall;// [maps][HW]
    const int32_t *map_scal;// [maps][MRTS_MAP_SCALARS]
    int G, HW, W, H;
    int nmaps;              // map templates (1: every game's terrain is map 0's)
    int nsp, nsp_games, max_steps, obs_float, partial_obs;
    const int64_t *actions; // [N][HW][7]
    const int32_t *src;     // [N][HW]
    void *obs;              // [N][HW][P]
    double *raw_reward;     // [N][6]
    uint8_t *done;          // [N][6]
    int32_t *mask;          // [N][HW][78]: k_masks output; k_step / k_reset write the
    int32_t *src_out;       // [N][HW]      next tick's masks here when non-null
    // optional fused step_wait outputs (vec_env.py:1057): reward = raw @ rw
    // (float64, k = 0..5 in order; channels 1..5 zeroed when !shaping) and done[:,0]
    double *reward;         // [N] or null
    uint8_t *done0;         // [N] or null (torch.bool storage)
    double rw[6];
    int shaping;
    // device bots (mrts_bots.hip): bot game b = game nsp_games + b
    const int32_t *bot_ai;  // [Gb] MRTS_AI_* of player 1
    const int32_t *bot_ai0; // [Gb] MRTS_AI_* of player 0 in bot-vs-bot games, -1 = the agent
    int4 *aa;               // [Gb][2][HW][2] AbstractionLayerAI.actions per bot player
    int32_t *botpa;         // [Gb][2][HW] bot PlayerActions, cell | code << 16; null = none
    int nbot_active;        // bot players (either side) whose AI is not passiveAI
    const int32_t *bot_games; // k_bot: decide only for these games (device list), null = every bot game
    int bot_ngames;
    int fuse_bots;          // k_step: wave 0 of each bot game's workgroup decides the next tick's bot actions
    int game_offset;        // global index of game 0 (a shard of a larger batch): keys the bots' RNG
    int early_bot;          // fused k_step: the bot may start beside phase A (mrts_engine_early_bot_ok for this size)
    const uint8_t *parked;  // [G] 1 = parked (mrts_park_games): no tick, no masks / bots, zero outputs at
                            // reset; null while no game was ever parked
};
__device__ __forceinline__ bool game_parked(const EngineParams &p, int g) { return p.parked && p.parked[g]; }

// The step kernel's argument: the engines of one launch and the grid's segments
// (workgroups seg_block[k] .. seg_block[k + 1] - 1 run games seg_game[k].. of
// engine e[seg_member[k]]).
#define MRTS_STEP_GROUP_MAX 4
struct StepGroup {
    EngineParams e[MRTS_STEP_GROUP_MAX];
    int seg_block[2 * MRTS_STEP_GROUP_MAX + 1];
    int seg_member[2 * MRTS_STEP_GROUP_MAX];
    int seg_game[2 * MRTS_STEP_GROUP_MAX];
    int nseg;
};

extern "C" {
hipError_t mrts_engine_reset(const EngineParams *p, hipStream_t s, const int32_t *games, const int32_t *maps, int count);
hipError_t mrts_engine_masks(const EngineParams *p, hipStream_t s);
hipError_t mrts_engine_outputs(const EngineParams *p, hipStream_t s);
hipError_t mrts_engine_step(const EngineParams *p, hipStream_t s);
hipError_t mrts_engine_step_group(const EngineParams *ps, int n, hipStream_t s, int bots_first);
size_t mrts_engine_group_lds_bytes(int HW, int W, int fused, int NT, int partial);
int mrts_engine_step_nt(int HW, int fused);
hipError_t mrts_engine_bots(const EngineParams *p, hipStream_t s);
hipError_t mrts_engine_raw_obs(const EngineParams *p, hipStream_t s, int32_t *raw);
hipError_t mrts_engine_sample(const int32_t *mask, int n, int hw, int env0, uint64_t seed, uint32_t step, int64_t *act, hipStream_t s);
hipError_t mrts_engine_sample_src(const int32_t *mask, const int32_t *src, int n, int hw, int env0, uint64_t seed, uint32_t step,
                                  int64_t *act, hipStream_t s);
hipError_t mrts_engine_sample_src_group(const mrts_sample_seg *segs, int nseg, uint64_t seed, uint32_t step, hipStream_t s);
hipError_t mrts_engine_render(const EngineParams *p, hipStream_t s, int game, int map, int size, uint8_t *rgb);
size_t mrts_engine_lds_bytes(int HW, int W);
size_t mrts_engine_bot_lds_bytes(int HW, int W);
size_t mrts_engine_fused_lds_bytes(int HW, int W, int partial);
int mrts_engine_early_bot_ok(int HW, int W);
}
#endif
