// mrts_bots.hip -- k_bot: the device-side scripted opponents (gym_microrts/microrts_ai.py)
// as their own launch, one wavefront per bot game; the bot logic itself is in
// mrts_bots.h (shared with the bot-fused k_step, mrts_engine.hip).
//
// Launched before k_step when the decisions of the tick are not already there:
// every step without fusion (bot-vs-bot games, or mrts_set_bot_fusion(h, 0)),
// and after resets with fusion (the fused k_step decides the NEXT tick's bot
// actions at the end of each step; a reset state needs them decided afresh).
#include "mrts_bots.h"

namespace mrts {
namespace bots {

// blockIdx.y = the bot's player: 1 = ai2 (every bot env), 0 = ai1 of a bot-vs-bot
// game (MicroRTSBotVecEnv); both see the same pre-issue state.  With a game list
// (p.bot_games), block i decides for game p.bot_games[i] if it is a bot game.
__global__ __launch_bounds__(BT) void k_bot(EngineParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int player = gridDim.y == 2 ? (int)blockIdx.y : 1;
    int b = blockIdx.x;
    if (p.bot_games) {
        b = p.bot_games[blockIdx.x] - p.nsp_games;
        if (b < 0) return;   // a selfplay game
    }
    if (game_parked(p, p.nsp_games + b)) return;
    bot_game<false>(p, b, player, smem);
}

}  // namespace bots
}  // namespace mrts

extern "C" {
hipError_t mrts_engine_bots(const EngineParams* p, hipStream_t s) {
    const int nb = p->bot_games ? p->bot_ngames : p->G - p->nsp_games;
    if (nb <= 0 || p->nbot_active == 0) return hipSuccess;
    hipLaunchKernelGGL(mrts::bots::k_bot, dim3(nb, p->bot_ai0 ? 2 : 1), dim3(mrts::bots::BT),
                       mrts::bots::bot_lds_bytes(p->HW, p->W), s, *p);
    return hipGetLastError();
}
size_t mrts_engine_bot_lds_bytes(int HW, int W) { return mrts::bots::bot_lds_bytes(HW, W); }
}
