"""Parity against the reference's SECOND build: seq_functions.cpp at -O3 (oracle/_ref/libref_seq_o3.so).

The pin is the FMA-contracted build (oracle/Makefile: -O2 -mfma -ffp-contract=fast), whose every
``sum += a*b`` (seq_functions.cpp:61, :82) is an fmaf chain -- what the reference's CUDA kernels
compute under nvcc's default contraction, and what the HIP path reproduces bit for bit
(tests/test_gpu_parity.py).  At -O3 GCC vectorises the products without FMA (vmulps + in-order
vaddss), so the unfused build rounds every product once more.  tests/golden/ref_o3.npz
(tests/golden/make_golden.py make_o3) holds that build's end states; here the fp32 path -- the
oracle restatement on the CPU, the HIP path on the GPU -- is held to:

  * z within 1e-6 norm-relative of the -O3 build at every K (100, 1000 and the C4 265 / 450);
  * y within 1e-6 at K = 100 (main.cu:87's N_v) and at the C4 265 / 450;
  * y at K = 1000 against the RECORDED bound Y_BOUND_1000 (measured 9.25e-5 on battery_c1,
    7.97e-5 on battery_10x4, 8.3e-7 on synth_small): the dual iterate of the battery problems is
    ill-conditioned and the two roundings drift apart, so 1e-6 does not hold there.
The C4 bound for y at 450 is 2e-6 (measured 8.8e-7 on these 16 instances; the round-4 review saw
1.21e-6 on other C4 instances).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN_SETS, f32_inputs, load_golden

Z_TOL = 1e-6
Y_TOL = 1e-6
Y_BOUND_1000 = 1.5e-4   # recorded: max 9.25e-5 (battery_c1)
Y_BOUND_C4_450 = 2e-6   # recorded: max 8.8e-7 here, 1.21e-6 seen elsewhere


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def y_bound(K):
    return Y_TOL if K <= 450 else Y_BOUND_1000


def o3():
    return load_golden("ref_o3")


def _oracle_fixed(oracle, ML, M, G, g, L, K):
    MGneg, GL, pD = oracle.scale(ML, G, g, L)
    if M.ndim == 1:
        z, y, _, _ = oracle.solve_f32(np.zeros(ML.shape[0]), np.zeros(ML.shape[1]), ML, M, G, g, K, L, 0.0)
        return z, y
    Z, Y, _, _ = oracle.solve_batch_f32(np.zeros(M.shape), np.zeros(g.shape), MGneg, M, GL,
                                        oracle.scale_vec(g, L), K, L, 0.0)
    return Z, Y


@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("K", [100, 1000])
def test_oracle_vs_o3_build_golden_sets(oracle, name, K):
    ML, M, G, g, L = f32_inputs(load_golden(name))
    d = o3()
    z, y = _oracle_fixed(oracle, ML, M, G, g, L, K)
    assert rel(z, d[f"{name}_z_{K}"]) <= Z_TOL
    assert rel(y, d[f"{name}_y_{K}"]) <= y_bound(K)


@pytest.mark.parametrize("K", [265, 450])
def test_oracle_vs_o3_build_c4_instances(oracle, K):
    d = o3()
    Z, Y = _oracle_fixed(oracle, d["c4_ML"], d["c4_M"], d["c4_G"], d["c4_g"], d["c4_L"], K)
    for i in range(Z.shape[0]):
        assert rel(Z[i], d[f"c4_z_{K}"][i]) <= Z_TOL
        assert rel(Y[i], d[f"c4_y_{K}"][i]) <= (Y_TOL if K == 265 else Y_BOUND_C4_450)


def test_y_bound_is_needed_at_1000(oracle):
    """The recorded bound is not slack: at K = 1000 the battery y is past 1e-6 from the -O3 build
    although the fp32 path equals the FMA build (the reference's CUDA arithmetic) bit for bit."""
    ML, M, G, g, L = f32_inputs(load_golden("battery_c1"))
    _, y = _oracle_fixed(oracle, ML, M, G, g, L, 1000)
    assert 1e-5 < rel(y, o3()["battery_c1_y_1000"]) <= Y_BOUND_1000


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["stream", "resident", "panel"])
@pytest.mark.parametrize("name", GOLDEN_SETS)
@pytest.mark.parametrize("K", [100, 1000])
def test_hip_vs_o3_build_golden_sets(gpu, kernel, name, K):
    from test_gpu_parity import run_gpu
    ML, M, G, g, L = f32_inputs(load_golden(name))
    d = o3()
    z, y, st, _ = run_gpu(ML, M, G, g, L, K, kernel=kernel)
    assert st["kernel"] == kernel and st["iterations"] == K
    assert rel(z, d[f"{name}_z_{K}"]) <= Z_TOL
    assert rel(y, d[f"{name}_y_{K}"]) <= y_bound(K)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [265, 450])
def test_hip_vs_o3_build_c4_instances(gpu, K):
    from test_gpu_parity import run_gpu
    d = o3()
    Z, Y, st, _ = run_gpu(d["c4_ML"], d["c4_M"], d["c4_G"], d["c4_g"], d["c4_L"], K)
    assert st["iterations"] == K
    for i in range(Z.shape[0]):
        assert rel(Z[i], d[f"c4_z_{K}"][i]) <= Z_TOL
        assert rel(Y[i], d[f"c4_y_{K}"][i]) <= (Y_TOL if K == 265 else Y_BOUND_C4_450)
