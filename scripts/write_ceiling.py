"""Steady-state HBM write ceiling for the bench loop's byte pattern (MI355X).

Back-to-back torch fills (each launch starts while the previous one's dirty tail
is still in the 256 MB MALL), HIP-event timed over many iterations:
  * fill 948.4 MB (k_step's algorithmic bytes at 16x16 / 8192 envs) alone, repeated;
  * fill 948.4 MB then fill 117.4 MB (the sampler's int64 actions), repeated —
    the byte pattern of one bench step.
  python scripts/write_ceiling.py
"""
import json

import torch


def timed(fn, iters=60, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3   # us per iteration


def main():
    step_b, samp_b = 948428800, 8192 * 256 * 7 * 8
    big = torch.empty(step_b // 4, dtype=torch.int32, device="cuda")
    act = torch.empty(samp_b // 8, dtype=torch.int64, device="cuda")
    out = {}
    t = timed(lambda: big.fill_(1))
    out["fill_step_bytes_repeated"] = {"us": round(t, 1), "TB/s": round(step_b / t / 1e6, 3)}
    t = timed(lambda: (big.fill_(1), act.fill_(2)))
    out["fill_step_then_actions"] = {"us": round(t, 1), "TB/s": round((step_b + samp_b) / t / 1e6, 3)}
    t1 = timed(lambda: act.fill_(2))
    out["fill_actions_repeated"] = {"us": round(t1, 1), "TB/s": round(samp_b / t1 / 1e6, 3)}
    big2 = torch.empty(step_b // 4, dtype=torch.int32, device="cuda")
    t = timed(lambda: big2.copy_(big))
    out["copy_step_bytes"] = {"us": round(t, 1), "TB/s_rw": round(2 * step_b / t / 1e6, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
