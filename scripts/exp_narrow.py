"""Experiment builds only (never the product library): copy microrts-py_amd/csrc to DEST and
cut the step / reset / mask dispatch down to the 16x16 workgroup (NT = 256), 29 planes and
float obs, so one engine object compiles in ~1 min instead of ~10.  Other map sizes,
partial observability and int32 obs then fail loudly (hipErrorInvalidValue from dispatch).

  python scripts/exp_narrow.py DEST [--sgpr N] [--vgpr N]
    --sgpr / --vgpr: add amdgpu_num_sgpr / amdgpu_num_vgpr to k_step (register budget A/B)
"""
import argparse
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "microrts-py_amd", "csrc")


def sub(s, a, b):
    assert a in s, a[:70]
    return s.replace(a, b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dest")
    ap.add_argument("--sgpr", type=int, default=0)
    ap.add_argument("--vgpr", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0, help="__launch_bounds__(NT, waves per SIMD) on k_step")
    a = ap.parse_args()
    if os.path.exists(a.dest):
        shutil.rmtree(a.dest)
    shutil.copytree(SRC, a.dest, ignore=shutil.ignore_patterns("build", "*.o"))
    p = os.path.join(a.dest, "mrts_engine.hip")
    s = open(p).read()
    s = sub(s, """    if (kind == 2 && p.fuse_bots) return step_nt(p.HW, true) == 128 ? launch_all<128>(p, kind, s, games, maps, count)
                                                                      : launch_all<256>(p, kind, s, games, maps, count);
    if (p.HW <= 64) return launch_all<64>(p, kind, s, games, maps, count);
    if (p.HW <= 128) return launch_all<128>(p, kind, s, games, maps, count);
    return launch_all<256>(p, kind, s, games, maps, count);""",
            """    if (p.HW <= 128 || p.partial_obs || !p.obs_float) return hipErrorInvalidValue;   // narrowed experiment build
    return launch_all<256>(p, kind, s, games, maps, count);""")
    for pp, ot in (("31", "float"), ("31", "int32_t"), ("29", "int32_t")):
        s = s.replace(f"k_reset<NT, {pp}, {ot}>", "k_reset<NT, 29, float>")
        s = s.replace(f"k_step<NT, {pp}, {ot}, true>", "k_step<NT, 29, float, true>")
        s = s.replace(f"k_step<NT, {pp}, {ot}>", "k_step<NT, 29, float>")
    s = sub(s, """    if (NT == 64) hipLaunchKernelGGL(mrts::k_raw<64>, dim3(p->G), dim3(64), sh, s, *p, raw);
    else if (NT == 128) hipLaunchKernelGGL(mrts::k_raw<128>, dim3(p->G), dim3(128), sh, s, *p, raw);
    else hipLaunchKernelGGL(mrts::k_raw<256>, dim3(p->G), dim3(256), sh, s, *p, raw);""",
            """    if (NT != 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mrts::k_raw<256>, dim3(p->G), dim3(256), sh, s, *p, raw);""")
    if a.sgpr or a.vgpr or a.waves:
        attr = ""
        if a.sgpr:
            attr += f" __attribute__((amdgpu_num_sgpr({a.sgpr})))"
        if a.vgpr:
            attr += f" __attribute__((amdgpu_num_vgpr({a.vgpr})))"
        lb = f"NT, {a.waves}" if a.waves else "NT"
        s = sub(s, "__global__ __launch_bounds__(NT) void k_step(EngineParams p) {",
                f"__global__ __launch_bounds__({lb}){attr} void k_step(EngineParams p) {{")
    open(p, "w").write(s)
    print("narrowed", a.dest)


if __name__ == "__main__":
    main()
