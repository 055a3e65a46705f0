"""The N-API addon (packages/merge-tree-native): the Node/TypeScript host binding of the C ABI."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "packages", "merge-tree-native")
ADDON = os.path.join(PKG, "build", "mte_native.node")

node = shutil.which("node")
pytestmark = pytest.mark.skipif(node is None, reason="node not installed")


def ensure_built():
    if not os.path.exists(ADDON):
        subprocess.run(["make", "-s", "-C", PKG], check=True)


def test_addon_exports_cpu():
    ensure_built()
    r = subprocess.run([node, os.path.join(PKG, "test", "exports.test.js")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "exports ok" in r.stdout


@pytest.mark.gpu
def test_addon_replay_gpu_matches_oracle():
    import ctypes

    from fluidframework_amd import mte
    from oracle import replay_batch

    ensure_built()
    r = subprocess.run([node, os.path.join(PKG, "test", "parity.gpu.js")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    eng = mte.Engine(0)
    eng.generate(2, 8, 500, n_clients=8, seed=3)
    batch = eng.export_batch()
    ops, cks, st = replay_batch(ctypes.addressof(batch), 0, 8, threads=4)
    assert out["ops"] == ops
    assert [int(c) for c in out["checksums"]] == cks
    assert out["interleaved_reads"] > 10
