"""The cutoff kernel's chunk plan (gpmdm_amd/csrc/common.h) checked on the host: the same
inline functions the kernel and the likelihood finish evaluate, compiled by hipcc into a host
program (tests/host/cutoff_plan_check.cpp; no HIP call, so it runs without a GPU).  CPU only."""
import shutil
import subprocess
from pathlib import Path

import pytest

from conftest import ROOT

HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if Path("/opt/rocm/bin/hipcc").exists() else None)


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_cutoff_chunk_plan(tmp_path):
    exe = tmp_path / "cutoff_plan_check"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", f"-I{ROOT / 'gpmdm_amd' / 'csrc'}",
           f"-I{ROOT / 'include'}", str(ROOT / "tests" / "host" / "cutoff_plan_check.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-3000:] + r.stderr[-3000:]
