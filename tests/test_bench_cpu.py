"""bench.py's host-side pieces that need no GPU: the sustained-rate phase (timing bookkeeping around a stub
solve) and the per-configuration flags a child measurement run receives."""
import argparse
import os
import sys
import time

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, REPO)
    import bench as b

    return b


def test_sustained_phase_runs_the_step_for_its_budget(bench):
    calls = []

    def solve():
        calls.append(1)
        time.sleep(0.004)
        return None, None

    args = argparse.Namespace(sustain_seconds=0.05)
    out = bench.sustain(args, solve, lambda: None, 0.01, 1, 128, torch.device("cpu"))
    assert out["steps"] == 5 == len(calls)  # budget / the timed step time, same count on every rank
    assert out["seconds"] >= 0.02 and out["value"] == pytest.approx(128 * 5 / out["seconds"], rel=5e-2)
    assert out["unit"] == "problems/s" and "not the headline" in out["note"]


def test_child_runs_skip_the_sustained_phase(bench):
    args = bench.parse(["--batch", "256", "--views", "16", "--points", "4096", "--no-distortion"])
    assert args.sustain_seconds == 10.0  # the default run carries the phase
    argv = bench._config_argv(args)
    assert "--no-distortion" in argv and "4096" in argv
    child = bench._child_argv(args)  # what live_traffic runs under rocprofv3 --pmc
    assert child[child.index("--sustain-seconds") + 1] == "0"
    assert "--no-live-counters" in child
    assert child[child.index("--steps") + 1] == "1" and child[child.index("--cpu-sample") + 1] == "0"
    assert child[-len(argv):] == argv  # the same configuration
    again = bench.parse(child[2:])  # and it parses back to this configuration
    assert (again.batch, again.views, again.points, again.no_distortion) == (256, 16, 4096, True)
    assert again.sustain_seconds == 0 and again.no_live_counters


def test_status_percentiles(bench):
    st = torch.zeros((100, 4), dtype=torch.int32)
    st[:, 2] = torch.arange(100)
    out = bench.status_percentiles(st)
    assert out["evaluations"]["max"] == 99 and out["evaluations"]["p50"] == pytest.approx(49.5)
    assert out["steps"]["max"] == 0 and set(out) == {"steps", "evaluations", "trials"}
