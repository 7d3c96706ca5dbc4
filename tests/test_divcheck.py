"""The FMA-corrected pivot division of the patch kernels' LLT solves (option patch_fdiv, llt_rcp in
ofdis_kernels.hip) against IEEE division: tools/divcheck_l.c on 6.4e9 (numerator, pivot) pairs of the range the
kernels take the fast form in (0 mismatches expected), and the checker's own sensitivity (a reciprocal one ulp
off must be caught)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "divcheck_l.c")


def _build(tmp_path, src_text=None):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = SRC
    if src_text is not None:
        src = str(tmp_path / "dc.c")
        with open(src, "w") as f:
            f.write(src_text)
    exe = str(tmp_path / "divcheck_l")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-mfma", "-o", exe, src, "-lm"], check=True)
    return exe


def _run(exe):
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    counts = [int(l.split(",")[1].split()[0]) for l in r.stdout.splitlines() if l.startswith("part")]
    return r.returncode, counts, r.stdout


def test_pivot_division_exact(tmp_path):
    rc, bad, out = _run(_build(tmp_path))
    assert len(bad) == 3 and rc == 0 and bad == [0, 0, 0], out


def test_checker_catches_a_wrong_reciprocal(tmp_path):
    text = open(SRC).read().replace("y = 1.0f / L;", "y = nextafterf(1.0f / L, 0.0f);")
    rc, bad, out = _run(_build(tmp_path, text))
    assert rc != 0 and sum(bad) > 0, out
