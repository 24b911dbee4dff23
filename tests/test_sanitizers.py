"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
§5: the reference runs `go test -race`; the C++ host runtime here gets the
sanitizers).  Builds the product DER parser (minbft_amd/csrc/der.cpp) with
the fuzz driver tests/csrc/der_fuzz.cpp using g++ and runs it over random
and mutated encodings; any sanitizer report fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_der_parser_asan_ubsan(tmp_path):
    exe = tmp_path / "der_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "minbft_amd", "csrc", "der.cpp"),
           os.path.join(ROOT, "tests", "csrc", "der_fuzz.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    for seed in (1, 2, 3):
        p = subprocess.run([str(exe), "150000", str(seed)], capture_output=True, text=True,
                           timeout=300, env=env)
        assert p.returncode == 0, p.stderr[-4000:]
        assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
        assert p.stdout.startswith("iterations 150000 parsed ")
