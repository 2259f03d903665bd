"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 sanitizers; host code only — GPU
sanitizers are not available on the pool): the product's host half of the topological loss
(`csrc/w2_host.cpp`: octsam_w2_host / octsam_topo_host, `csrc/api.cpp`) and the oracle's C persistence,
driven by `tests/sanitize/host_driver.cpp` on random, tied, checkerboard and empty inputs, with the W_q cost
checked against a brute-force assignment for tiny diagrams."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    obj = tmp_path / "cubical_ph.o"
    subprocess.run(["gcc", "-std=c11", *san, "-c", os.path.join(ROOT, "oracle", "cubical_ph.c"), "-o", str(obj)],
                   check=True)
    exe = tmp_path / "host_driver"
    subprocess.run(["g++", "-std=c++17", *san, os.path.join(ROOT, "tests", "sanitize", "host_driver.cpp"),
                    os.path.join(ROOT, "dilabhelmholtzoct_amd", "csrc", "w2_host.cpp"),
                    os.path.join(ROOT, "dilabhelmholtzoct_amd", "csrc", "api.cpp"), str(obj), "-o", str(exe)],
                   check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
