"""CustomAllReduce._apply_calibration on synthetic rank-max tables (no GPU): the crossovers the
``auto`` policy and the TP registered-output cutoff use (a table without two-shot
entries must not push every large message onto one-shot)."""

import types

import pytest

from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import CustomAllReduce

KB, MB = 1 << 10, 1 << 20


def _car(world):
    c = object.__new__(CustomAllReduce)
    c.comm = types.SimpleNamespace(world_size=world)
    c.oneshot_max, c.auto_max = 256 * KB, 8 * MB
    return c


def _row(n, **us):
    return {"bytes": n, "us": us}


def test_standard_table():
    c = _car(8)
    c._apply_calibration([
        _row(4 * KB, rccl=30.0, oneshot=9.0, twoshot=11.0, reg_pull=10.0, reg_push=10.5),
        _row(512 * KB, rccl=40.0, oneshot=20.0, twoshot=18.0, reg_pull=15.0, reg_push=16.0),
        _row(16 * MB, rccl=120.0, oneshot=400.0, twoshot=150.0, reg_pull=110.0, reg_push=None),
        _row(64 * MB, rccl=420.0, oneshot=None, twoshot=500.0, reg_pull=430.0, reg_push=None),
    ])
    assert c.oneshot_max == 4 * KB          # two-shot ahead from 512 KiB
    assert c.auto_max == 512 * KB           # RCCL ahead of both staged forms at 16 MiB
    assert c.reg_max == 16 * MB             # registered pull still ahead at 16 MiB
    assert c.calibration["agreed"] == "rank-max" and c.calibration["world"] == 8


def test_missing_twoshot_rows_stop_the_oneshot_scan():
    """Two-shot measured at the small sizes but not at a larger one (e.g. a size that is no
    multiple of W vectors): one-shot must not be extended past what was compared."""
    c = _car(6)
    c._apply_calibration([
        _row(4 * KB, rccl=30.0, oneshot=9.0, twoshot=11.0),
        _row(64 * KB, rccl=35.0, oneshot=10.0, twoshot=None),
        _row(16 * MB, rccl=120.0, oneshot=100.0, twoshot=None),
    ])
    assert c.oneshot_max == 4 * KB


def test_twoshot_never_ran_keeps_oneshot_everywhere_it_wins():
    """Two-shot failed its check everywhere (None at every size): one-shot is the only staged
    form, so it is used up to the largest size calibrated."""
    c = _car(3)
    c._apply_calibration([
        _row(4 * KB, rccl=30.0, oneshot=9.0, twoshot=None),
        _row(16 * MB, rccl=120.0, oneshot=100.0, twoshot=None),
    ])
    assert c.oneshot_max == 16 * MB and c.auto_max == 16 * MB


@pytest.mark.parametrize("world", [2, 3, 5, 6, 7, 8])
def test_calibration_sizes_admit_twoshot_for_every_world(world):
    """The sizes calibrate() times are rounded to W 16-byte vectors, so two-shot's divisibility
    condition holds at every size for every W (powers of two fail it at W = 3, 5, 6, 7)."""
    from distributed_llm_backend_benchmark_amd.parallel.custom_allreduce import CALIB_SIZES

    for n in CALIB_SIZES:
        m = n - n % (16 * world)
        assert m > 0 and m % (8 * 2 * world) == 0
