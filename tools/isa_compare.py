"""Compare the gfx950 instruction streams of two builds of libgpmdm_hip.so kernel by kernel.

    python tools/isa_compare.py OLD.so NEW.so [kernel-substring]

Kernel-argument offsets (s_load immediates, struct-size multipliers) and the PC-relative
offset right after s_getpc_b64 (the address of a __constant__ table, which moves when other
data of the code object changes) are normalised, so a change to the argument structs or to
unrelated constant data alone reads as "same".  Used to show that splitting the A/B
laboratory out of gp_tile.h left every production tile instantiation's code unchanged
(profiles/r03/isa_compare_lab_split.txt)."""
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/llvm/bin")


def code_objects(lib, tmp):
    fat = Path(tmp) / "fat.bin"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(Path(tmp) / "x.o")],
                   check=True, capture_output=True)
    b = fat.read_bytes()
    magic, out, pos = b"__CLANG_OFFLOAD_BUNDLE__", [], 0
    while (i := b.find(magic, pos)) >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if triple.endswith("gfx950") and size:
                co = Path(tmp) / f"co{len(out)}.o"
                co.write_bytes(b[i + off:i + off + size])
                out.append(co)
        pos = i + 1
    return out


def kernels(lib):
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            asm = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                                 text=True).stdout
            fn, after_pc = None, False
            for line in asm.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
                if m:
                    fn = m.group(1)
                    out[fn] = []
                    continue
                if fn and line.strip():
                    ins = re.sub(r"\s+", " ", line.split("//")[0].strip())
                    if ins.startswith(("s_load", "s_mul")) or (after_pc and ins.startswith("s_add_u32")):
                        ins = re.sub(r"0x[0-9a-f]+|\b\d+\b", "N", ins)
                    after_pc = ins.startswith("s_getpc_b64")
                    out[fn].append(ins)
    return out


def main():
    old, new = kernels(sys.argv[1]), kernels(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    same = diff = 0
    for k in sorted(new):
        if sub not in k:
            continue
        if k not in old:
            print(f"new only: {k}")
        elif old[k] == new[k]:
            same += 1
        else:
            diff += 1
            print(f"DIFFERENT: {k} ({len(old[k])} vs {len(new[k])} instructions)")
    gone = [k for k in old if sub in k and k not in new]
    for k in gone:
        print(f"old only: {k}")
    print(f"{same} kernels with identical instruction streams, {diff} different, {len(gone)} removed")


if __name__ == "__main__":
    main()
