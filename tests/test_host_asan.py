"""Host sanitizers on the C ABI's host-side code: the model
descriptor validation and the MFMA-fragment image packing of gpmdm_model_create
(gpmdm_amd/csrc/host_image.h, the same header capi_model.hip compiles) built with
-fsanitize=address,undefined and driven by tests/asan/host_image_check.cpp.  CPU only."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_image_packing_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_image_check"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT / 'gpmdm_amd' / 'csrc'}", f"-I{ROOT / 'include'}",
           str(ROOT / "tests" / "asan" / "host_image_check.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # verify_asan_link_order=0: the sanitizer runtime need not be first in the library list
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-3000:] + r.stderr[-3000:]
