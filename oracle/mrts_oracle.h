/*
 * mrts_oracle.h -- CPU restatement of the MicroRTS engine + JNI vector client.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU surrogate).  The product path (libmicrorts_amd.so) never
 * links or calls it.
 *
 * What it restates (the Java lives in the absent submodule
 * gym_microrts/microrts -> adFrej/MicroRTS-KG):
 *   rts.GameState.{issueSafe,issue,cycle,getVectorObservation}, rts.UnitAction
 *   .{execute,resourceUsage,ETA,fromVectorAction}, rts.PlayerAction
 *   .{fromVectorAction,fillWithNones}, rts.ResourceUsage.consistentWith,
 *   rts.units.Unit.getUnitActions, rts.units.UnitTypeTable() (VERSION_ORIGINAL,
 *   MOVE_CONFLICT_RESOLUTION_CANCEL_BOTH), ai.reward.* and
 *   tests.JNIGridnetVecClient.{reset,gameStep,getMasks}, as called from
 *   /root/reference/gym_microrts/envs/vec_env.py:261-282, 1001-1057, 1091-1101.
 * Parity anchors: reference tests/test_observation.py, tests/test_mask.py,
 * tests/test_reward.py (ported in repo tests/test_oracle_kat.py) and the
 * _encode_obs golden vectors in tests/golden/.  Engine rules beyond those
 * fixtures are UNPINNED (choices in DESIGN.md §4).
 *
 * The data structures deliberately follow the Java object model (a unit list in
 * insertion order, a LinkedHashMap of unit -> action assignment) rather than
 * the GPU's cell-major SoA, so GPU==oracle agreement is a check between two
 * independent formulations.
 */
#ifndef MRTS_ORACLE_H
#define MRTS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OVec OVec;

/* A map as PhysicalGameState.load would see it (XML order preserved). */
typedef struct {
    int32_t width, height;
    const uint8_t *terrain;  /* [height*width], 1 = wall                      */
    int32_t player_res[2];
    int32_t num_units;
    const int32_t *units;    /* [num_units][6]: type, player, x, y, resources, hitpoints */
} OMap;

/* AI ids for bot envs (gym_microrts/microrts_ai.py names). */
enum { OAI_PASSIVE = 0, OAI_WORKER_RUSH = 1, OAI_LIGHT_RUSH = 2, OAI_RANDOM_BIASED = 3, OAI_COAC = 4,
       OAI_PO_WORKER_RUSH = 5, OAI_PO_LIGHT_RUSH = 6, OAI_PO_HEAVY_RUSH = 7, OAI_PO_RANGED_RUSH = 8,
       OAI_RANDOM = 9 };

OVec *ovec_create(int num_selfplay, int num_bot, int max_steps, int partial_obs,
                  const OMap *maps, int num_maps, const int32_t *game_map,
                  const int32_t *bot_ai, const int32_t *bot_ai0 /* NULL or -1: agent is p0 */);
void ovec_destroy(OVec *v);
int ovec_num_envs(const OVec *v);

/* JNIGridnetVecClient.reset([0]*N) */
void ovec_reset(OVec *v);
/* Reset one game (map cycling, vec_env.py:1038-1056). */
void ovec_reset_game(OVec *v, int game, int map_id);
/* JNIGridnetVecClient.getMasks(0) -> int[N][H*W][79] (channel 0 = source unit). */
void ovec_get_masks(OVec *v, int32_t *masks);
/* JNIGridnetVecClient.gameStep: actions [N][H*W][7] (the python-side action
 * tensor), source_mask [N][H*W] from the last get_action_mask selects the rows
 * (vec_env.py:968-984).  Outputs raw rewards [N][6] and dones [N][6]. */
void ovec_step(OVec *v, const int64_t *actions, const int32_t *source_mask,
               double *reward, uint8_t *done);
/* Response.observation: raw planes int[N][P_raw][H][W] (P_raw = 6, or 7 with
 * partial obs) as returned after the last reset/step. */
void ovec_raw_obs(OVec *v, int32_t *raw);
/* vec_env.py:311-321 (_encode_obs, prior_mode none): raw -> one-hot
 * int32 [N][H][W][P] */
void ovec_encode_obs(const int32_t *raw, int n, int h, int w, int partial_obs, int32_t *out);

/* Debug / differential hooks: per-game scalars and the unit list. */
int ovec_game_time(const OVec *v, int game);
void ovec_game_resources(const OVec *v, int game, int32_t *res2);
/* Cell-major dump: [H*W][8] = type(-1 empty), player, hp, resources,
 * action type (-1 none), action param, action done time, action issue time. */
void ovec_dump_cells(const OVec *v, int game, int32_t *out);

/* Counter-based random masked-action sampler shared with the GPU bench
 * sampler (hello_world.py:27-64 semantics: per cell and component, uniform
 * over mask-valid entries; uniform over all entries when none is valid).
 * masks: [N][H*W][78] (channels 1..78 of getMasks), actions out [N][H*W][7]. */
void ovec_sample_actions(const int32_t *masks78, int n, int hw, int env0, uint64_t seed,
                         uint32_t step, int64_t *actions);   /* env0: global index of row 0's env */

/* CPU baseline of bench.py: `steps` whole env-steps (masks, sampler, step,
 * obs encode) with OpenMP over envs; see mrts_oracle.c. */
void ovec_bench_steps(OVec *v, int steps, uint64_t seed, uint32_t step0, int32_t *masks79, int64_t *act, int32_t *src,
                      double *reward, uint8_t *done, int32_t *obs);

/* Trajectory statistics (test diagnostics, not part of the restated API): event
 * counts summed over every game since creation, resets included.
 * [OEV_CANCEL_BOTH] issue's same-cycle conflicts (both actions -> NONE),
 * [OEV_INCONSISTENT] issue's conflicts with an older assignment (new -> NONE),
 * [OEV_PRODUCED + 7 * player + type] units produced (executed), by type,
 * [OEV_HITS + player] attacks that hit a unit, [OEV_KILLS + player] units killed. */
enum { OEV_CANCEL_BOTH = 0, OEV_INCONSISTENT = 1, OEV_PRODUCED = 2, OEV_HITS = 16, OEV_KILLS = 18, OEV_N = 20 };
void ovec_event_counts(const OVec *v, int64_t *out);

#ifdef __cplusplus
}
#endif
#endif
