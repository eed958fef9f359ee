"""Randomised parity (tests/fuzz_util.py): random shapes, batch sizes, kernels, fixed-N and
Algorithm-1 modes, test periods, warm starts, schedule options, host / device memory and
repeated solves on one handle, each checked bit for bit (z*, y*, iteration counts) against the
oracle on a sample of instances.  A fixed seed here; tools/fuzz_parity.py runs many more."""
from __future__ import annotations

import json

import numpy as np
import pytest

import fuzz_util

SEED = 20261018
CASES = 12


def test_fuzz_cases_are_deterministic_and_valid():
    a = [fuzz_util.draw_case(np.random.default_rng(SEED + i)) for i in range(50)]
    b = [fuzz_util.draw_case(np.random.default_rng(SEED + i)) for i in range(50)]
    assert json.dumps(a) == json.dumps(b)
    for c in a:
        assert 1 <= c["n"] <= 260 and 1 <= c["m"] <= 260 and c["batch"] >= 1
        assert c["kernel"] != "resident" or max(c["n"], c["m"]) <= 208
        assert c["kernel"] != "panel" or c["shared"]
        assert (c["tol"] > 0) == (c["N"] == 2000)
        assert not c["f64"] or (c["shared"] and c["kernel"] != "resident")


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(CASES))
def test_fuzz_parity(gpu, oracle, i):
    cfg = fuzz_util.draw_case(np.random.default_rng(SEED + i))
    r = fuzz_util.run_case(cfg, oracle)
    assert r["ok"], f"{json.dumps(cfg)}: {r['why']}"
    assert r["checked"] >= min(cfg["batch"], 2) * cfg["solves"]


FLAT_CASES = 6


def test_flat_fuzz_cases_are_valid():
    for i in range(50):
        c = fuzz_util.draw_flat_case(np.random.default_rng(SEED + i))
        assert 1 <= c["n_u"] <= 16 and 1 <= c["Nh"] <= 60 and c["kernel"] in ("auto", "panel", "stream")


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(FLAT_CASES))
def test_flat_fuzz_parity(gpu, oracle, i):
    cfg = fuzz_util.draw_flat_case(np.random.default_rng(SEED + 100 + i))
    r = fuzz_util.run_flat_case(cfg, oracle)
    assert r["ok"], f"{json.dumps(cfg)}: {r['why']}"


VALUE_CASES = 6


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(VALUE_CASES))
def test_value_fuzz_parity(gpu, oracle, i):
    cfg = fuzz_util.draw_value_case(np.random.default_rng(SEED + 200 + i))
    r = fuzz_util.run_value_case(cfg, oracle)
    assert r["ok"], f"{json.dumps(cfg)}: {r['why']}"


LOOP_CASES = 4


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(LOOP_CASES))
def test_closed_loop_fuzz_parity(gpu, oracle, i):
    cfg = fuzz_util.draw_loop_case(np.random.default_rng(SEED + 300 + i))
    r = fuzz_util.run_loop_case(cfg, oracle)
    assert r["ok"], f"{json.dumps(cfg)}: {r['why']}"


HEAVY_CASES = 2


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(HEAVY_CASES))
def test_heavy_fuzz_parity(gpu, oracle, i):
    """C3 / C4-shaped phased solves (planner, compaction, duo finisher) with random schedule options;
    the four longest instances of every solve are among those checked."""
    cfg = fuzz_util.draw_heavy_case(np.random.default_rng(SEED + 400 + i))
    r = fuzz_util.run_case(cfg, oracle)
    assert r["ok"], f"{json.dumps(cfg)}: {r['why']}"


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(4))
def test_step_entry_points_fuzz(gpu, oracle, i):
    r = fuzz_util.run_steps_case(SEED + 500 + i, oracle)
    assert r["ok"], r["why"]
