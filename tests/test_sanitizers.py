"""Host-code sanitizers (VERDICT r1 hygiene): the oracle and the bitboard CPU
engine (bitboard.hpp compiled for the host) built with
-fsanitize=address,undefined into one executable (tests/host/san_main.cpp)
and driven through every exported entry point for N = 4..16.  GPU sanitizers
are not available on the pool; this covers the host-compiled code."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_and_bitboard_engine_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_main")
    san = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all",
           "-static-libasan", "-static-libubsan"]
    obj = str(tmp_path / "oracle.o")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-c", "-o", obj,
                           os.path.join(ROOT, "oracle", "othello_oracle.c")] + san)
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Wextra", "-Wno-unknown-pragmas", "-o", exe,
                           os.path.join(ROOT, "tests", "host", "san_main.cpp"),
                           os.path.join(ROOT, "oracle", "cpu_bitboard.cpp"), obj] + san)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "clean" in r.stdout
