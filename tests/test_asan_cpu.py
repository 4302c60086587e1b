"""`make asan`: the host-side C++ (shape -> kernel geometry, config selection,
LDS / split-K / slab sizing, the 32-bit offset guards) under AddressSanitizer +
UndefinedBehaviorSanitizer, driven over every model's shapes and the oversize
rejection paths by csrc/host_check.cpp.  CPU only: the .hip files
are compiled host-only, no kernel is launched."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) and shutil.which("make")),
                                reason="needs hipcc and make")


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    out = tmp_path_factory.mktemp("asan")
    r = subprocess.run(["make", "-s", "asan", f"ASAN_DIR={out}"], cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "0 failed" in r.stdout, r.stdout[-2000:]
    return os.path.join(out, "host_check"), r.stdout


def test_make_asan_runs_clean(host_check):
    _, out = host_check
    line = [ln for ln in out.splitlines() if ln.startswith("host_check:")][-1]
    checks = int(line.split()[1])
    assert checks > 10000, line


@pytest.mark.parametrize("kind,marker", [("asan", "AddressSanitizer"),
                                         ("ubsan", "runtime error")])
def test_sanitizers_are_live(host_check, kind, marker):
    """A deliberate heap overflow / signed overflow must abort the same binary."""
    exe, _ = host_check
    r = subprocess.run([exe], env=dict(os.environ, DMP_ASAN_SELFTEST=kind), capture_output=True,
                       text=True, timeout=60)
    assert r.returncode != 0 and marker in r.stderr, r.stderr[-2000:]
