"""Code-generation guard (CPU): no production kernel in libgpmdm_hip.so stores more than 8
bytes from VGPRs in one instruction.

On gfx950 (ROCm 7.2) a 16-byte buffer store whose data registers the next instruction
refilled from LDS wrote a wrong low dword for 0.33% of the values; 8-byte stores of the
same registers were exact (tools/microbench/store_hazard.hip).  The ISA rule
this matches covers stores of more than 8 bytes followed by a write of their data VGPRs; the
compiler pads a VALU write behind such a store but not an LDS or memory return.  So every
production kernel stores through 8-byte (or narrower) stores, and this test disassembles the
built code objects and fails on any wider global / buffer / flat store.

Compiler-generated spill stores (``scratch_store_*``) fall under the same rule: a
default-shape kernel may not spill through stores wider than 8 bytes (only the opt-in 64x256
shape, GPMDM_TILE_SHAPE=1, does at d >= 7), and the default shapes do not spill at all for
d <= 12 (a spill in the K loop would also cost time).  The cutoff kernel (k_obs_cutoff,
obs_cutoff.h) keeps a few loop-invariant addresses in scratch at some d; none of its
scratch accesses may sit between its first and last MFMA (the K loops)."""
import re
import shutil
import struct
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "gpmdm_amd" / "libgpmdm_hip.so"
LLVM = Path("/opt/rocm/llvm/bin")
WIDE_STORE = re.compile(r"\b(buffer|global|flat)_store_(dwordx[34]|b96|b128)\b")
WIDE_SPILL = re.compile(r"\bscratch_store_(dwordx[34]|b96|b128)\b")
SPILL_STORE = re.compile(r"\bscratch_store_")
# kernels allowed a wide store: none
ALLOW_WIDE: set = set()


def _code_objects(tmp_path):
    """The gfx950 code objects of the library's offload bundles (.hip_fatbin)."""
    fat = tmp_path / "fat.bin"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(LIB), str(tmp_path / "x.o")],
                   check=True, capture_output=True)
    b = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], 0
    while (i := b.find(magic, pos)) >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if triple.endswith("gfx950") and size:
                co = tmp_path / f"co{len(out)}.o"
                co.write_bytes(b[i + off:i + off + size])
                out.append(co)
        pos = i + 1
    return out


SCRATCH = re.compile(r"\bscratch_(store|load)_")
MFMA = re.compile(r"\bv_mfma_")


def _stores_by_kernel(co):
    asm = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                         text=True).stdout
    wide, wspill, spill, fn = {}, {}, {}, None
    seq = {}                               # per kernel: "m" (MFMA) / "s" (scratch access) in order
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            fn = m.group(1)
            continue
        if WIDE_STORE.search(line):
            wide[fn] = wide.get(fn, 0) + 1
        if WIDE_SPILL.search(line):
            wspill[fn] = wspill.get(fn, 0) + 1
        if SPILL_STORE.search(line):
            spill[fn] = spill.get(fn, 0) + 1
        if MFMA.search(line):
            seq.setdefault(fn, []).append("m")
        elif SCRATCH.search(line):
            seq.setdefault(fn, []).append("s")
    in_loop = {f for f, q in seq.items() if "m" in q and "s" in "".join(q).strip("s")}
    return wide, wspill, spill, in_loop


def _tile_args(kernel: str):
    m = re.search(r"k_gp_tileILi(\d+)ELb([01])ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", kernel)
    return None if not m else tuple(int(x) for x in m.groups())


def _default_shape(kernel: str) -> bool:
    """A k_gp_tile instantiation a default model uses (capi_model.hip gpmdm_model_create: the
    observation GP 32x512 for d <= 12 / 64x512 above, dynamics 16x256 plus a wide image in
    the observation shape).  Template args: <d, dyn, VAR, NW, MT, NTW>."""
    m = re.search(r"k_gp_tileILi(\d+)ELb([01])ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", kernel)
    if not m:
        return True                       # every other kernel is production
    d, dyn, var, nw, mt, ntw = (int(x) for x in m.groups())
    shape = (nw, mt, ntw)
    obs = (4, 2, 8) if d <= 12 else (8, 4, 4)
    return shape == obs or (dyn == 1 and shape == (4, 1, 4))


@pytest.mark.skipif(not (LLVM / "llvm-objdump").exists() or not LIB.exists(), reason="ROCm llvm tools / library")
def test_no_wide_vgpr_stores_in_production_kernels(tmp_path):
    cos = _code_objects(tmp_path)
    assert cos, "no gfx950 code object found in libgpmdm_hip.so"
    wide, wspill, spill, in_loop = {}, {}, {}, set()
    for co in cos:
        w, ws, s, il = _stores_by_kernel(co)
        wide.update(w)
        wspill.update(ws)
        spill.update(s)
        in_loop |= il
    bad = {k: v for k, v in wide.items() if k not in ALLOW_WIDE}
    assert not bad, f"wide (>8-byte) stores in production kernels: {bad}"
    bad = {k: v for k, v in wspill.items() if _default_shape(k)}
    assert not bad, f"default-shape kernels spill through wide scratch stores: {bad}"
    bad = {k: v for k, v in spill.items() if _default_shape(k) and _tile_args(k) and _tile_args(k)[0] <= 12}
    assert not bad, f"default-shape kernels at d <= 12 spill: {bad}"
    cut = {k for k in spill if "k_obs_cutoff" in k}
    assert not {k for k in spill if not _tile_args(k)} - cut, "a non-tile kernel spills"
    assert not (cut & in_loop), f"the cutoff kernel spills inside its K loop: {cut & in_loop}"
