/*
 * microrts_amd.h -- C ABI of the MI355X-native vectorised MicroRTS engine
 * (libmicrorts_amd.so).
 *
 * This is the drop-in replacement for the FFI boundary the reference crosses
 * on every reset / step / get_action_mask: JPype -> Java
 * tests.JNIGridnetVecClient (constructed at
 * /root/reference/gym_microrts/envs/vec_env.py:259-271).  Plain pointers and
 * sizes only; no torch types.  Device buffers are allocated by the caller
 * (hipMalloc, or a torch tensor's data_ptr) and all work is enqueued on the
 * caller's hipStream_t, passed as `void *stream` (NULL = default stream).
 *
 * Ownership (reference: JNI path copies, shared-mem path aliases,
 * vec_env.py:1276-1283, 1331-1333): output buffers are written in place and
 * stay valid until the next call that writes them.
 *
 * Errors: every call returns MRTS_OK (0) or a negative MRTS_E* code, and
 * mrts_last_error() holds a message (the reference surfaces Java exceptions
 * through JPype; callers invoke e.printStackTrace(), ppo_gridnet.py:477-479).
 *
 * Threading: a handle is not thread-safe; one handle per device per process
 * (the reference runs one in-process JVM per process, vec_env.py:153-169).
 */
#ifndef MICRORTS_AMD_H
#define MICRORTS_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRTS_OK 0
#define MRTS_EINVAL (-1)
#define MRTS_EIO (-2)
#define MRTS_EHIP (-3)
#define MRTS_ENOTIMPL (-4)
#define MRTS_ESTATE (-5)

/* Opponent ids for bot envs; names as in gym_microrts/microrts_ai.py:13-61. */
#define MRTS_AI_PASSIVE 0
#define MRTS_AI_WORKER_RUSH 1
#define MRTS_AI_LIGHT_RUSH 2
#define MRTS_AI_RANDOM_BIASED 3
#define MRTS_AI_COAC 4
#define MRTS_AI_PO_WORKER_RUSH 5
#define MRTS_AI_PO_LIGHT_RUSH 6
#define MRTS_AI_PO_HEAVY_RUSH 7
#define MRTS_AI_PO_RANGED_RUSH 8
#define MRTS_AI_RANDOM 9 /* randomAI = ai.RandomBiasedSingleUnitAI (microrts_ai.py:7-10) */
#define MRTS_AI_COUNT 10

#define MRTS_OBS_INT32 0
#define MRTS_OBS_FLOAT32 1

typedef struct mrts_vec mrts_vec;

/* Arguments of JNIGridnetVecClient(num_selfplay, num_bot, max_steps, rfs,
 * micrortsPath, mapPaths, ai2s, utt, partialObs) (vec_env.py:261-271).  The six
 * reward functions and the default UnitTypeTable are fixed (vec_env.py:172-195). */
typedef struct {
    int32_t num_selfplay_envs;   /* even; envs 2k/2k+1 are players 0/1 of game k */
    int32_t num_bot_envs;        /* envs num_selfplay + j play player 0 vs bot_ai[j] */
    int32_t max_steps;           /* JNIGridnetVecClient.maxSteps                     */
    int32_t partial_obs;         /* PartiallyObservableGameState (31 planes)         */
    int32_t num_maps;            /* map table: all maps share one height x width     */
    const char *const *map_paths;/* PhysicalGameState XML files (absolute paths)     */
    const int32_t *game_map;     /* [num_games] index into map_paths, NULL -> 0      */
    const int32_t *bot_ai;       /* [num_bot_envs] MRTS_AI_*, NULL -> passive        */
    int32_t obs_dtype;           /* MRTS_OBS_INT32 (reference dtype) or FLOAT32      */
    const int32_t *bot_ai0;      /* [num_bot_envs] MRTS_AI_* of player 0 (bot vs bot,
                                    MicroRTSBotVecEnv / JNIBotClient, vec_env.py:1104-1236),
                                    -1 = the agent plays player 0; NULL = all agent */
    int32_t game_offset;         /* global index of game 0 when this handle is one shard
                                    of a larger batch (one process per GPU): keys the
                                    random bots' streams so shard r's games play exactly
                                    as games [game_offset, game_offset + num_games) of
                                    one unsharded run; 0 otherwise                    */
    int32_t map_capacity;        /* map template slots (>= num_maps; 0 -> num_maps):
                                    room for maps added later with mrts_add_map      */
} mrts_config;

typedef struct {
    int32_t height, width;
    int32_t num_envs, num_games;
    int32_t obs_planes;          /* 29, or 31 with partial obs                       */
    int32_t mask_channels;       /* 78 (getMasks' 79 minus the source channel)       */
    int32_t action_components;   /* 7                                                */
    size_t workspace_bytes;      /* device bytes mrts_bind_workspace needs           */
} mrts_info_t;

/* new JNIGridnetVecClient(...): parses the map XMLs, validates the config. */
int mrts_create(const mrts_config *cfg, mrts_vec **out);
int mrts_info(const mrts_vec *h, mrts_info_t *info);
/* Attach caller-owned device memory of mrts_info().workspace_bytes (game state
 * + map templates) and upload the maps on `stream`. */
int mrts_bind_workspace(mrts_vec *h, void *dev_workspace, void *stream);

/* JNIGridnetVecClient.reset(players) (vec_env.py:279): every game back to its
 * map; obs [N][H][W][planes] (int32 or float32 per obs_dtype). */
int mrts_reset(mrts_vec *h, void *stream, void *obs);

/* JNIGridnetVecClient.getMasks(0) (vec_env.py:1097): mask [N][H*W][78] int32
 * (channels 1..78) and source [N][H*W] int32 (channel 0). */
int mrts_get_masks(mrts_vec *h, void *stream, int32_t *mask, int32_t *source);

/* Bind device mask outputs (the zero-copy form of the reference's shared-memory
 * client, Client(..., obsBuf, maskBuf, actionBuf, 0), vec_env.py:1276-1283,
 * 1310-1324): from now on mrts_reset, mrts_step, mrts_step_weighted and
 * mrts_reset_games also write getMasks(0) of the state they leave behind --
 * the bytes a following mrts_get_masks would write -- into mask [N][H*W][78]
 * int32 and source [N][H*W] int32, in the same kernel pass.  `source` may be
 * the buffer mrts_step reads its rows from (each game reads its own rows
 * before it rewrites them).  NULL, NULL unbinds. */
int mrts_bind_mask_outputs(mrts_vec *h, int32_t *mask, int32_t *source);

/* Bot fusion (default on).  A bot's getAction(1, gs) reads only the state
 * before the tick (JNIGridnetClient.gameStep: bot decisions, then issueSafe(p0),
 * issueSafe(p1), cycle).  With fusion, mrts_step's kernel decides the NEXT
 * tick's bot actions for every bot game in the same pass -- one wavefront of the
 * game's workgroup runs the bot on the state it has just stored while the other
 * wavefronts stream the observations and masks -- instead of a separate bot
 * kernel at the start of the next step; mrts_reset / mrts_reset_games decide
 * them for the games they reset.  Outputs are identical either way.  Applies
 * when no env has a bot as player 0 (MicroRTSBotVecEnv), the map has more than
 * 64 cells and its two LDS regions fit one workgroup (160 KB); on = 0 launches the bot kernel at every step. */
int mrts_set_bot_fusion(mrts_vec *h, int32_t on);

/* step_async + JNIGridnetVecClient.gameStep (vec_env.py:968-984, 1002):
 * actions [N][H*W][7] int64 (device), source [N][H*W] int32 = the source
 * channel of the last mrts_get_masks (selects the rows, vec_env.py:974).
 * Outputs: obs, raw_reward [N][6] float64 (the six reward functions), done
 * [N][6] uint8.  Finished games auto-reset (terminal reward/done reported). */
int mrts_step(mrts_vec *h, void *stream, const int64_t *actions, const int32_t *source,
              void *obs, double *raw_reward, uint8_t *done);

/* Response.observation of the JNI client (vec_env.py:279-280, 1002-1003, 1035):
 * GameState.getVectorObservation per env, int32 [N][P_raw][H][W], P_raw = 6
 * (hp, resources, owner 1 = self / 2 = opponent, type id + 1, action type,
 * terrain) + 1 visibility plane with partial obs.  The unencoded form of the
 * obs mrts_reset / mrts_step write; for callers that keep the reference's own
 * python _encode_obs. */
int mrts_get_raw_obs(mrts_vec *h, void *stream, int32_t *raw);

/* reward_weight and reward_shaping of MicroRTSGridModeVecEnv (vec_env.py:102-103,
 * 1003-1004, 1057), used by mrts_step_weighted.  Host array of 6 doubles. */
int mrts_set_reward_weight(mrts_vec *h, const double *weight6, int32_t reward_shaping);

/* mrts_step + the step_wait reduction fused into the same kernel
 * (vec_env.py:1003-1004, 1057): reward [N] float64 = raw_reward @ weight
 * (k = 0..5 in order, round-to-nearest, no FMA; channels 1..5 taken as 0 when
 * reward_shaping is off) and done0 [N] uint8 = done[:, 0]. */
int mrts_step_weighted(mrts_vec *h, void *stream, const int64_t *actions, const int32_t *source, void *obs,
                       double *raw_reward, uint8_t *done, double *reward, uint8_t *done0);

/* One step of several engines -- the map-size buckets of one mixed batch --
 * equivalent to mrts_step (io[i].reward == NULL) or mrts_step_weighted on each
 * hs[i] in order on `stream`.  Replaces the sequence of
 * JNIGridnetVecClient.gameStep calls that one reference vec env per map size
 * makes (vec_env.py:148-150: one size per env; vec_env.py:986-1003: gameStep),
 * so that engines whose kernels share planes, obs dtype and bot fusion run in
 * one kernel launch instead of one each.  policy: MRTS_GROUP_SEPARATE (one
 * launch per engine), MRTS_GROUP_MERGE_FIT (merge members that still fit
 * >= 4 workgroups per CU at the launch's LDS size; larger maps keep their own
 * launch), MRTS_GROUP_MERGE_ALL (every compatible member), | MRTS_GROUP_BOTS_FIRST
 * (bot games start before selfplay games in the merged grid).  Outputs are the
 * same bytes whatever the policy.  1 <= n <= MRTS_STEP_GROUP_MAX, each handle once,
 * all on the device that runs `stream`.  Errors: the message is on the failing
 * member's handle and on hs[0].  Not atomic: when launch l fails with MRTS_EHIP the
 * members of earlier launches have stepped and the others have not. */
#define MRTS_STEP_GROUP_MAX 4
#define MRTS_GROUP_SEPARATE 0
#define MRTS_GROUP_MERGE_FIT 1
#define MRTS_GROUP_MERGE_ALL 2
#define MRTS_GROUP_BOTS_FIRST 4
typedef struct mrts_step_io {
    const int64_t *actions;
    const int32_t *source;
    void *obs;
    double *raw_reward;
    uint8_t *done;
    double *reward;   /* NULL: mrts_step's outputs only */
    uint8_t *done0;
} mrts_step_io;
int mrts_step_group(mrts_vec *const *hs, int32_t n, void *stream, const mrts_step_io *io, int32_t policy);

/* The launches mrts_step_group(hs, n, ..., policy) would make now: launch_of[i] =
 * the launch (0 ..) engine i runs in, *launches = their number.  No reference
 * counterpart (an engine-internal schedule, for profiling and tests). */
int mrts_step_group_plan(mrts_vec *const *hs, int32_t n, int32_t policy, int32_t *launch_of, int32_t *launches);

/* Map cycling (vec_env.py:1038-1056): reset `count` games (host arrays) onto
 * the given map indices and rewrite their envs' obs; parked games play again. */
int mrts_reset_games(mrts_vec *h, void *stream, const int32_t *games, const int32_t *maps, int32_t count, void *obs);

/* Park `count` games (host array): they stop ticking -- mrts_step, mrts_get_masks
 * and the bots skip them -- and their envs' obs (and bound mask / source) rows
 * are written as zeros now; reward / done rows are left to the caller.
 * mrts_reset_games restarts a parked game on a map (mrts_reset keeps it parked
 * and writes its zeros again).  Map cycling across map sizes
 * (MicroRTSSizeCyclingVecEnv): a game lives in one engine per size and plays in
 * one of them. */
int mrts_park_games(mrts_vec *h, void *stream, const int32_t *games, int32_t count, void *obs);

/* JNIGridnetVecClient.clients[i].mapPath = path / .selfPlayClients[j].mapPath =
 * path (vec_env.py:1044, 1051): the Java client re-reads the map file at its next
 * reset.  Here the map is loaded into a free template slot (config map_capacity)
 * and its index returned, for mrts_reset_games; a path already in the table
 * returns its existing index.  Same height x width as the handle's maps. */
int mrts_add_map(mrts_vec *h, void *stream, const char *path, int32_t *index);

/* Random masked action sampler of hello_world.py:27-64 on the device
 * (Philox4x32-10 keyed by seed, counter = (cell, env0 + env, step)): env0 is the
 * global index of row 0's env, so a shard draws the actions of its slice of
 * one larger batch.  Not a reference entry point: the bench's stand-in policy. */
int mrts_sample_actions(void *stream, const int32_t *mask, int32_t num_envs, int32_t hw, int32_t env0, uint64_t seed,
                        uint32_t step, int64_t *actions);

/* Same stream and output as mrts_sample_actions, given the source channel too
 * (num_envs * hw must stay below 2^31 - 64: MRTS_EINVAL otherwise):
 * mask rows of cells whose source is 0 are all zero (getMasks), so only the
 * rows of source cells are read.  Every row's 7 components are still written. */
int mrts_sample_actions_src(void *stream, const int32_t *mask, const int32_t *source, int32_t num_envs, int32_t hw,
                            int32_t env0, uint64_t seed, uint32_t step, int64_t *actions);

/* mrts_sample_actions_src over up to MRTS_SAMPLE_GROUP_MAX batches at once (the map-size
 * buckets of one mixed batch) in ONE launch: segment k's actions are exactly those
 * mrts_sample_actions_src(stream, seg.mask, seg.source, seg.num_envs, seg.hw, seg.env0,
 * seed, step, seg.actions) writes.  Each segment: num_envs * hw below 2^31 - 256,
 * actions 16-byte aligned; MRTS_EINVAL otherwise.  The bench's stand-in policy. */
#define MRTS_SAMPLE_GROUP_MAX 4
typedef struct mrts_sample_seg {
    const int32_t *mask;     /* [num_envs][hw][78] */
    const int32_t *source;   /* [num_envs][hw] */
    int32_t num_envs, hw, env0;
    int64_t *actions;        /* [num_envs][hw][7] */
} mrts_sample_seg;
int mrts_sample_actions_src_group(void *stream, const mrts_sample_seg *segs, int32_t nseg, uint64_t seed, uint32_t step);

/* Per-game rollout statistics, host int32 out[num_games][MRTS_GAME_STATS]:
 * game time (ticks since the game's last reset; the reference's gs.getTime()),
 * env steps of the episode, steps since creation, and three never-reset
 * counters -- ticks whose ready actions executed in order on one lane (attacks
 * or a shared resource pile), action rows issued on the ordered one-lane path,
 * auto-resets.  Synchronises the stream.  Introspection only (bench.py reports
 * the episode phases and serial work its timed window covered). */
#define MRTS_GAME_STATS 6
int mrts_game_stats(mrts_vec *h, void *stream, int32_t *out);

/* render("rgb_array") (vec_env.py:1075-1084): the game of `env` drawn into a
 * device frame rgb [size][size][3] uint8 (RGB; the reference returns 640 x 640).
 * Drawing rules: DESIGN.md §4c (the Java panel is absent; parity unpinned). */
int mrts_render(mrts_vec *h, void *stream, int32_t env, uint8_t *rgb, int32_t size);

/* Env-state checkpoint (no reference counterpart; SURVEY.md §5 "env-state
 * checkpoint"): the games' whole state -- cells, scalars, map templates, the
 * device bots' abstract actions and PlayerActions, parked flags, and the host-side
 * mirrors -- copied into / out of a caller device buffer of mrts_state_bytes(h)
 * bytes (256-byte aligned).  mrts_save_state synchronises the stream.
 * mrts_load_state restores a snapshot of the same configuration and map table
 * into this handle -- same env split, obs layout, game offset, max_steps, bots (both
 * players) and map templates, checked by a fingerprint in the snapshot's header; MRTS_EINVAL
 * otherwise, before anything but the fixed header is read -- and writes the restored state's obs
 * into `obs` (and its next-tick masks into the bound mask outputs), as mrts_reset
 * does for a fresh state; stepping on from it repeats the saved run bit for bit.
 * The reward weights and shaping flag (mrts_set_reward_weight) are host settings the
 * caller may change between steps: they are not in the snapshot and not checked. */
size_t mrts_state_bytes(const mrts_vec *h);
int mrts_save_state(mrts_vec *h, void *stream, void *dst);
int mrts_load_state(mrts_vec *h, void *stream, const void *src, void *obs);

/* Engine invariant violations recorded on the device (OR over games). */
int mrts_error_flags(mrts_vec *h, void *stream, int32_t *flags_out);

/* Diagnostics of the bot-fused step kernel for a map size (no device work, no
 * handle): 1 = the bot may start beside the output words' build (its LDS writes
 * and that phase's reads / writes are disjoint, checked from both carves),
 * 0 = fusable but the bot waits for that phase, -1 = no bot fusion for this
 * size (fused LDS over 160 KB, or a bot LDS over the 64 KB mrts_create allows).  No reference counterpart (an engine-internal schedule). */
int mrts_fused_layout_ok(int32_t width, int32_t height);

/* UnitTypeTable JSON as rts.units.UnitTypeTable.toJSON / sendUTT()
 * (vec_env.py:276).  Valid for the lifetime of the handle. */
const char *mrts_utt_json(const mrts_vec *h);

const char *mrts_last_error(const mrts_vec *h);
void mrts_destroy(mrts_vec *h);
const char *mrts_version(void);

#ifdef __cplusplus
}
#endif
#endif
