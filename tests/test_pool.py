"""The plan build's parallel_for (csrc/common.h): persistent workers, one job
at a time, nested and concurrent calls served by fresh threads, exceptions
rethrown, a forked child starting its own workers.  Host C++ only."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_parallel_for_workers(tmp_path):
    exe = str(tmp_path / "pool_check")
    inc = os.path.join(ROOT, "superlu_dist_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I" + inc,
                    "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "pool_check.cpp"), "-o", exe], check=True)
    env = dict(os.environ, SLU_PLAN_THREADS="8")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_parallel_for_workers_thread_sanitizer(tmp_path):
    """The same checks under ThreadSanitizer: no data race in the hand-off."""
    exe = str(tmp_path / "pool_check_tsan")
    inc = os.path.join(ROOT, "superlu_dist_amd", "csrc")
    b = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=thread", "-I" + inc,
                        "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "cpp", "pool_check.cpp"), "-o", exe],
                       capture_output=True, text=True)
    if b.returncode != 0:
        pytest.skip("no ThreadSanitizer runtime: " + b.stderr[-300:])
    env = dict(os.environ, SLU_PLAN_THREADS="8", TSAN_OPTIONS="die_after_fork=0 halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr, \
        r.stdout + r.stderr[-3000:]
