"""Generate the committed golden vectors under tests/golden/ (run in the BUILD container only).

Sources of truth:
  * the reference's own CPU steps (Code/CUDA/FinalProject/src/seq_functions.cpp), compiled in
    place by ``make -C oracle ref`` into oracle/_ref/libref_seq.so and composed in the loop order
    of main.cu:160-175 (pyoracle.RefSeq) -> fp32 end states after K = 1, 10, 100 iterations and
    one-step known-answer vectors;
  * a numpy restatement of Code/MATLAB/acceldualgrad.m (tests/matlab_ref.py) -> fp64 end states;
  * our oracle (oracle/liboracle.so) for the Algorithm-1 (tol) runs, which the reference lacks.

Inputs are stored in float64; the fp32 path receives ``x.astype(np.float32)`` of them.
Usage:  python tests/golden/make_golden.py [--o3-only]
"""
from __future__ import annotations

import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gpu-dualgradient-mpc_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import matlab_ref  # noqa: E402
import pyoracle  # noqa: E402
from gpad_mpc import problems  # noqa: E402

STEP3_SRC = "/root/reference/Code/CUDA/FinalProject/build/step3"


def problem_set():
    return {
        "battery_c1": problems.battery_mpc(4, 10, seed=0),        # config C1: n=40, m=180
        "battery_10x4": problems.battery_mpc(10, 4),              # gpad.m:10 fixed x0, n=40, m=168
        "synth_small": problems.synthetic_qp(48, 80, seed=7),     # generic generator, n=48, m=80
    }


def make(name, qp, O, R):
    n, m = qp.n, qp.m
    f32 = lambda a: np.asarray(a, np.float64).astype(np.float32)  # noqa: E731
    ML, M, G, g, L = f32(qp.ML), f32(qp.M), f32(qp.G), f32(qp.g), np.float32(qp.L)
    MGneg, GL, pD = O.scale(ML, G, g, L)
    th, be = O.schedule_f32(100)
    out = dict(ML=qp.ML, M=qp.M, G=qp.G, g=qp.g, L=np.float64(qp.L), H=qp.H, q=qp.q,
               theta100=th, beta100=be)
    z0 = np.zeros(n, np.float32)
    y0 = np.zeros(m, np.float32)
    for K in (1, 10, 100):
        z, y = R.solve(z0, y0, MGneg, M, GL, pD, th, be, K)
        out[f"ref_z_{K}"], out[f"ref_y_{K}"] = z, y
    # warm-started run (z0, y0 nonzero) -- exercises the y_0 = y_{-1} initialisation
    rng = np.random.default_rng(123)
    zw = rng.normal(0, 0.1, n).astype(np.float32)
    yw = np.abs(rng.normal(0, 0.1, m)).astype(np.float32)
    z, y = R.solve(zw, yw, MGneg, M, GL, pD, th, be, 50)
    out.update(warm_z0=zw, warm_y0=yw, ref_warm_z_50=z, ref_warm_y_50=y)
    # one-step known-answer vectors (8a..8d) on a random state
    ym1 = np.abs(rng.normal(0, 0.2, m)).astype(np.float32)
    yv = np.abs(rng.normal(0, 0.2, m)).astype(np.float32)
    zm1 = rng.normal(0, 0.2, n).astype(np.float32)
    beta, theta = np.float32(be[57]), np.float32(th[52])
    w = R.step1(yv, ym1, beta)
    zh = R.step2(MGneg, w, M)
    z = R.step3(theta, zm1, zh)
    yp = R.step4(GL, w, pD, zh)
    out.update(kat_y=yv, kat_ym1=ym1, kat_zm1=zm1, kat_beta=beta, kat_theta=theta, kat_w=w,
               kat_zhat=zh, kat_z=z, kat_yp1=yp)
    # fp64 MATLAB restatement (acceldualgrad.m) after 100 iterations
    if qp.H is not None:
        _, zm, ym = matlab_ref.acceldualgrad(qp.H, qp.q, qp.G, qp.g, 1, 100, L=qp.L)
        out["matlab_z_100"], out["matlab_y_100"] = zm, ym
        _, zp, yp_ = matlab_ref.acceldualgrad(qp.H, qp.q, qp.G, qp.g, 1, 100, kind="paper", L=qp.L)
        out["matlab_paper_z_100"], out["matlab_paper_y_100"] = zp, yp_
    # Algorithm 1 (tol = 1e-4, K = 10) from the oracle
    z, y, it, conv = O.solve_f32(z0, y0, ML, M, G, g, 5000, L, 1e-4, 10)
    out.update(tol_z=z, tol_y=y, tol_iters=np.int32(it), tol_conv=np.int32(conv))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: n={n} m={m} L={qp.L:.6g} tol-iters={it}")


def write_reference_datafile(path, d, flipped):
    """A main.cu:29-67 data file written with plain numpy formatting (independent of the
    libgpad writer, so the reader is tested against a file it did not produce)."""
    n = d["M_G"].shape[0]
    with open(path, "w") as fh:
        fh.write(f"{d['n_u']} {d['N']} {d['m']} {len(d['theta'])} {d['L']:.8e}\n")
        mg = d["M_G"].T if flipped else d["M_G"]          # flipped: M_G[j*n + i]
        gl = d["G_L"].T if flipped else d["G_L"]          # flipped: G_L[j*m + i]
        for arr in (mg.reshape(-1), d["g_P"], gl.reshape(-1), d["p_D"], d["theta"], d["beta"]):
            fh.write(" ".join(f"{v:.8e}" for v in np.asarray(arr, np.float64)) + "\n")
    assert n == d["n_u"] * d["N"]


def make_datafile(O, R):
    """gpad.m's default battery (n = 3 cells, p = 4: n = 12, m = 56) as a reference data file,
    with the reference's own steps (RefSeq) run for N_v = 100 iterations on the file's values
    (what main.cu computes, on the CPU steps it mirrors)."""
    qp = problems.battery_mpc(3, 4, seed=5)
    L = np.float32(qp.L)
    f32 = lambda a: np.asarray(a, np.float64).astype(np.float32)  # noqa: E731
    MGneg, GL, pD = O.scale(f32(qp.ML), f32(qp.G), f32(qp.g), L)
    th, be = O.schedule_f32(120)
    d = dict(n_u=3, N=4, m=qp.m, L=float(L), M_G=MGneg, g_P=f32(qp.M), G_L=GL, p_D=pD,
             theta=th, beta=be)
    write_reference_datafile(os.path.join(HERE, "datafile_battery_3x4.txt"), d, flipped=False)
    write_reference_datafile(os.path.join(HERE, "datafile_battery_3x4_flipped.txt"), d, flipped=True)
    # values as read back by fscanf("%f") == strtof of the printed text
    rd = lambda a: np.array([np.float32(float(f"{v:.8e}")) for v in np.asarray(a, np.float64).reshape(-1)],  # noqa: E731
                            np.float32).reshape(np.shape(a))
    fd = {k: rd(d[k]) for k in ("M_G", "g_P", "G_L", "p_D", "theta", "beta")}
    z0 = np.zeros(qp.n, np.float32)
    y0 = np.zeros(qp.m, np.float32)
    z, y = R.solve(z0, y0, fd["M_G"], fd["g_P"], fd["G_L"], fd["p_D"], fd["theta"], fd["beta"], 100)
    np.savez_compressed(os.path.join(HERE, "datafile_battery_3x4.npz"), L=np.float32(rd(d["L"])),
                        ref_z_100=z, ref_y_100=y, **fd)
    print(f"datafile_battery_3x4: n={qp.n} m={qp.m}")


def make_flat(name, n_u, N, seed, O, R):
    """The reference's FLAT battery steps (seq_functions.cpp:5-43) on the flattened battery
    problem: end states after 1, 10, 100 iterations (reference's own steps, main_prof.cu loop),
    one-step KATs, an Algorithm-1 run (oracle), and the ENABLE_FLATTEN_MATRICES data file."""
    qp = problems.battery_mpc(n_u, N, seed=seed)
    MGf, GLf, L = problems.flatten_battery(qp, n_u, N)
    f32 = lambda a: np.asarray(a, np.float64).astype(np.float32)  # noqa: E731
    L32 = np.float32(L)
    MGf32, GLf32, gP = f32(MGf), f32(GLf), f32(qp.M)
    pD = O.scale_vec(f32(qp.g), L32)
    th, be = O.schedule_f32(100)
    n, m = qp.n, qp.m
    out = dict(MGf=MGf32, GLf=GLf32, gP=gP, pD=pD, L=L32, n_u=np.int32(n_u), N=np.int32(N),
               theta100=th, beta100=be)
    z0, y0 = np.zeros(n, np.float32), np.zeros(m, np.float32)
    for K in (1, 10, 100):
        z, y = R.solve_flat_c(z0, y0, MGf32, gP, GLf32, pD, n_u, th, be, K)
        out[f"ref_z_{K}"], out[f"ref_y_{K}"] = z, y
    rng = np.random.default_rng(7)
    w = np.abs(rng.normal(0, 0.2, m)).astype(np.float32)
    zh = rng.normal(0, 0.2, n).astype(np.float32)
    out.update(kat_w=w, kat_zh_in=zh, kat_zhat=R.step2_flat(MGf32, w, gP, n_u),
               kat_yp1=R.step4_flat(GLf32, w, pD, zh, n_u))
    z, y, it, conv = O.solve_flat_f32(z0, y0, MGf32, gP, GLf32, pD, n_u, 5000, L32, 1e-4)
    out.update(tol_z=z, tol_y=y, tol_iters=np.int32(it), tol_conv=np.int32(conv))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"{name}: n={n} m={m} tol-iters={it}")
    return out


def write_flat_datafile(path, d, n_u, N):
    """ENABLE_FLATTEN_MATRICES data file (main.cu:39-56): M_G N x m, G_L m x N, numpy-formatted."""
    with open(path, "w") as fh:
        fh.write(f"{n_u} {N} {d['GLf'].shape[0]} 100 {float(d['L']):.8e}\n")
        for arr in (d["MGf"].reshape(-1), d["gP"], d["GLf"].reshape(-1), d["pD"], d["theta100"], d["beta100"]):
            fh.write(" ".join(f"{v:.8e}" for v in np.asarray(arr, np.float64)) + "\n")


def make_closed_loop():
    """gpad.m:79-95 with n = 3 cells, p = 4, 40 samples, acceldualgrad's 100 iterations per
    step, fp64 (numpy restatement of the MATLAB): x, u trajectories."""
    n_u, N, steps = 3, 4, 40
    mats = problems.battery_matrices(n_u, N)
    x = np.random.default_rng(11).random(n_u) - 0.5           # gpad.m:14 (seeded)
    xs, us = [], []
    for _ in range(steps):
        f, A_i, b_i = problems.battery_constraints(mats, x, n_u, N)
        u, _, _ = matlab_ref.acceldualgrad(mats["H"], f, A_i, b_i, n_u, 100)
        xs.append(x.copy())
        us.append(u.copy())
        x = mats["A"] @ x + mats["B"] @ u                      # gpad.m:93
    np.savez_compressed(os.path.join(HERE, "closed_loop_battery_3x4.npz"), x0=xs[0],
                        xs=np.array(xs), us=np.array(us), x_final=x)
    print(f"closed_loop_battery_3x4: steps={steps}")


def make_o3(O):
    """End states from the reference's OTHER build, _ref/libref_seq_o3.so (seq_functions.cpp at
    -O3 -march=x86-64-v3: GCC vectorises the products, vmulps + in-order vaddss, no FMA; the build
    bench.py times as cpu_baseline).  The parity pin is the FMA build (libref_seq.so); these
    fixtures state how far the HIP path is from the unfused one (tests/test_o3_parity.py):
      * the golden sets at K = 100 (main.cu:87's N_v) and K = 1000, from zero;
      * 16 C4-generator instances (bench.make_shard, n = m = 200) at K = 265 (the C4 mean to eps)
        and K = 450 (its longest solves), their fp32 inputs stored with them."""
    R3 = pyoracle.RefSeq(pyoracle.REF_O3)
    R = pyoracle.RefSeq()
    f32 = lambda a: np.asarray(a, np.float64).astype(np.float32)  # noqa: E731
    out = {}
    for name, qp in problem_set().items():
        n, m = qp.n, qp.m
        ML, M, G, g, L = f32(qp.ML), f32(qp.M), f32(qp.G), f32(qp.g), np.float32(qp.L)
        MGneg, GL, pD = O.scale(ML, G, g, L)
        th, be = O.schedule_f32(1000)
        for K in (100, 1000):
            z, y = R3.solve(np.zeros(n, np.float32), np.zeros(m, np.float32), MGneg, M, GL, pD, th, be, K)
            out[f"{name}_z_{K}"], out[f"{name}_y_{K}"] = z, y
            zf, yf = R.solve(np.zeros(n, np.float32), np.zeros(m, np.float32), MGneg, M, GL, pD, th, be, K)
            print(f"{name} K={K}: |dz|/|z| {np.linalg.norm(z - zf) / np.linalg.norm(zf):.3g} "
                  f"|dy|/|y| {np.linalg.norm(y - yf) / np.linalg.norm(yf):.3g} (O3 vs FMA build)")
    sys.path.insert(0, ROOT)
    import bench
    ML, G, L, M, g = bench.make_shard(200, 200, 16, 0)
    ML, G, M, g, L = f32(ML), f32(G), f32(M), f32(g), np.float32(L)
    out.update(c4_ML=ML, c4_G=G, c4_M=M, c4_g=g, c4_L=L)
    MGneg, GL, _ = O.scale(ML, G, g[0], L)
    PD = O.scale_vec(g, L)
    th, be = O.schedule_f32(450)
    for K in (265, 450):
        Z = np.zeros((16, 200), np.float32)
        Y = np.zeros((16, 200), np.float32)
        Zf, Yf = Z.copy(), Y.copy()
        for i in range(16):
            Z[i], Y[i] = R3.solve(Z[i], Y[i], MGneg, M[i], GL, PD[i], th, be, K)
            Zf[i], Yf[i] = R.solve(Zf[i], Yf[i], MGneg, M[i], GL, PD[i], th, be, K)
        out[f"c4_z_{K}"], out[f"c4_y_{K}"] = Z, Y
        rz = np.linalg.norm(Z - Zf, axis=1) / np.linalg.norm(Zf, axis=1)
        ry = np.linalg.norm(Y - Yf, axis=1) / np.linalg.norm(Yf, axis=1)
        print(f"c4 K={K}: max |dz|/|z| {rz.max():.3g} max |dy|/|y| {ry.max():.3g} (O3 vs FMA build)")
    np.savez_compressed(os.path.join(HERE, "ref_o3.npz"), **out)


def main():
    if "--o3-only" in sys.argv:
        pyoracle.build(ref=True)
        make_o3(pyoracle.Oracle())
        return
    pyoracle.build(ref=True)
    O = pyoracle.Oracle()
    R = pyoracle.RefSeq()
    for name, qp in problem_set().items():
        make(name, qp, O, R)
    make_datafile(O, R)
    make_closed_loop()
    make_o3(O)
    make_flat("battery_flat_4x10", 4, 10, 0, O, R)
    d = make_flat("battery_flat_3x4", 3, 4, 5, O, R)
    write_flat_datafile(os.path.join(HERE, "datafile_battery_flat_3x4.txt"), d, 3, 4)
    # the reference's own step-3 known-answer files (data, copied verbatim)
    if os.path.isdir(STEP3_SRC):
        for k in range(1, 6):
            dst = os.path.join(HERE, "step3", str(k))
            os.makedirs(dst, exist_ok=True)
            for f in ("input.txt", "output.txt"):
                shutil.copyfile(os.path.join(STEP3_SRC, str(k), f), os.path.join(dst, f))
        print("step3 fixtures copied")


if __name__ == "__main__":
    main()
