"""GPU: the C++ host mirror of the Go API (go-crdt-playground_amd/host/crdt.hpp)
replays the reference's scenario tests on the device (tests/cpp/test_scenarios.cpp;
built by __graft_entry__.build()).  This process uses the ROCm runtime directly,
no PyTorch: the standalone path a Go/C++ caller takes."""

import os
import subprocess

import pytest

from helpers import ROOT

BIN = os.path.join(ROOT, "go-crdt-playground_amd", "host", "build", "test_scenarios")


@pytest.mark.gpu
@pytest.mark.parametrize("rank_ids", ["0", "1"])
def test_cpp_scenarios_on_gpu(rank_ids):
    """rank_ids=1: every document takes the mirror's hash-collision fallback
    (ids = the keys' ranks in string order) instead of 64-bit hash ids."""
    assert os.path.exists(BIN), "build() first"
    env = dict(os.environ, CRDT_HOST_RANK_IDS=rank_ids)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=100, env=env)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 0 failure(s)" in r.stdout


def test_cpp_mirror_builds():
    assert os.path.exists(BIN)
