// mrts_layout.h -- device-resident state layout of the MI355X MicroRTS engine.
//
// One GAME = one rts.GameState (a selfplay pair of envs 2k/2k+1 shares one game;
// a bot env owns one).  Game state is cell-major: one 16-byte record per grid
// cell (the unit standing on it + that unit's pending UnitActionAssignment), so
// a workgroup loads/stores a whole 16x16 game with one coalesced dwordx4 per lane.
//
//   cells  int4  [G][HW]  .x unit word  .y unit insertion index (pgs.units order)
//                         .z action word .w issue sequence (LinkedHashMap order)
//   genv   int32 [G][GENV_WORDS]
//   bot games only (mrts_bots.hip): aa int4 [Gb][2][HW][2] (each bot player's
//   abstract actions, LinkedHashMap order), botpa int32 [Gb][2][HW] (cell | code << 16)
//   maps   per map: template cells int4 [HW], terrain u8 [HW], scalars int32 [4]
//
// Unit word   : bits 0-3 type+1 (0 = empty) | 4-5 owner+1 (0 = none/resource)
//               | 6-15 hit points | 16-31 carried / pile resources
// Action word : 0 = no assignment | bits 0-2 action type+1 | 3-8 parameter
//               (direction 0-3, or attack offset index 0-48 of the 7x7 grid)
//               | 9-11 produced unit type | 12-31 (issue time + ETA) + 1
// Sequence    : issue_time << 13 | player << 12 | rank-in-PlayerAction
#ifndef MRTS_LAYOUT_H
#define MRTS_LAYOUT_H
#include <stdint.h>

#define MRTS_NTYPES 7
#define MRTS_ATTACK_GRID 7
#define MRTS_MASK_CH 78      /* channels returned by get_action_mask */
#define MRTS_MASK_BITS 79    /* + source-unit channel 0 (getMasks) */
#define MRTS_MAX_HW 4096
#define MRTS_MAX_TIME 500000 /* 19-bit issue time in the sequence word */

/* per-game scalars; AA_N..NPA are used by bot games only:
 *   AA_N  entries of the bot's AbstractionLayerAI.actions list (mrts_bots.hip)
 *   TICKS steps since creation (never reset; bot RNG counter)
 *   NPA   entries of the bot PlayerAction handed from k_bot to k_step
 * rollout statistics, never reset (mrts_game_stats):
 *   SERIAL   ticks whose ready set executed in order on one lane (attacks, shared piles)
 *   ORDERED  action rows issued on the ordered (one-lane) path: the agent's and the device bots' rows
 *            still CAND after the lane-parallel pass (k_step compacts both kinds into one list)
 *   EPISODES auto-resets (gameover or max_steps) */
enum { MRTS_G_TIME = 0, MRTS_G_RES0, MRTS_G_RES1, MRTS_G_NEXT_UID, MRTS_G_STEPS, MRTS_G_MAP, MRTS_G_ERR, MRTS_G_AA_N,
       MRTS_G_TICKS, MRTS_G_NPA, MRTS_G_AA_N0, MRTS_G_NPA0, MRTS_G_SERIAL, MRTS_G_ORDERED, MRTS_G_EPISODES,
       MRTS_GENV_WORDS = 16 };   /* *0: player-0 bot (bot vs bot) */
enum { MRTS_M_RES0 = 0, MRTS_M_RES1, MRTS_M_NUNITS, MRTS_M_PAD, MRTS_MAP_SCALARS };

/* error bits recorded in genv[MRTS_G_ERR] (invariant violations) */
enum { MRTS_ERR_PRODUCE_OCCUPIED = 1, MRTS_ERR_MOVE_OCCUPIED = 2, MRTS_ERR_TIME_OVERFLOW = 4, MRTS_ERR_BOT_OVERFLOW = 8 };

#endif
