#!/usr/bin/env python3
"""Scan gfx950 assembly for a VMEM store whose data VGPRs are rewritten by
VALU before two wait states have passed (tools only; nothing imports this).

Found with tools/overlap_lab.hip (profiles/r03_overlap_lab.log): hipcc (ROCm
7.2) emitted `buffer_store_dwordx4 v[206:209] ...` directly followed by
`v_mov_b32 v208, v202`, and when other waves were issuing on the same SIMD
the store wrote the NEW value of v208:v209 in some lanes (lanes 12-15 of each
16-lane group, i.e. the data dwords the store read last). `s_nop 1` after
the store (two wait states) made every result bitwise again; the compiler
itself pads global_store_dwordx4 (FLAT) with such a wait but not the raw
buffer stores.

Usage: python3 tools/store_hazard_scan.py file.s|lib.so [...]
(a .so: its gfx950 code object is taken from the .hip_fatbin offload bundle
and disassembled with llvm-objdump)
A line is reported when a store of more than 8 bytes (dwordx2 excluded) is
followed, within the next two issued instructions (s_nop k counts k + 1),
by a v_* instruction whose destination overlaps the store's data registers.
Control flow is followed in text order only (labels are skipped).
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

STORE = re.compile(r"^\s*(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\s+(.*)$")
VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok):
    m = VREG.fullmatch(tok.strip())
    if not m:
        return set()
    if m.group(1):
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return {int(m.group(3))}


def operands(rest):
    return [t.strip() for t in rest.split(",")]


def code_object(so_path, arch="gfx950"):
    """The device code object for `arch` inside a HIP shared library."""
    data = open(so_path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    at = data.find(magic)
    while at >= 0:
        n = struct.unpack_from("<Q", data, at + 24)[0]
        off = at + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24: off + 24 + ts].decode()
            off += 24 + ts
            if triple.endswith(arch) and es:
                return data[at + eo: at + eo + es]
        at = data.find(magic, at + 1)
    raise RuntimeError(f"no {arch} code object in {so_path}")


def disassemble(so_path):
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "lib.co")
        open(co, "wb").write(code_object(so_path))
        out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--mcpu=gfx950", co], check=True,
                             capture_output=True, text=True).stdout
    lines = []
    for ln in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", ln)
        lines.append(m.group(1) + ":" if m else ln.split("//")[0])
    return lines


def scan(path):
    lines = open(path).read().splitlines() if path.endswith(".s") else disassemble(path)
    func = "?"
    hits = []
    for i, ln in enumerate(lines):
        if re.match(r"^[A-Za-z_][\w.$]*:", ln) and not ln.startswith(".L"):
            func = ln.split(":")[0]
        m = STORE.match(ln)
        if not m:
            continue
        ops = operands(m.group(3))
        # buffer_store: vdata is operand 0; global/flat/scratch_store: vaddr, vdata
        data = regs(ops[0]) if m.group(1) == "buffer" else regs(ops[1] if len(ops) > 1 else "")
        waits = 0
        j = i + 1
        while j < len(lines) and waits < 2:
            t = lines[j].split(";")[0].strip()
            j += 1
            if not t or t.endswith(":") or t.startswith("."):
                continue
            if t.startswith("s_nop"):
                waits += int(t.split()[1], 0) + 1
                continue
            if t.startswith("v_"):
                parts = t.split(None, 1)
                if len(parts) > 1:
                    dst = regs(operands(parts[1])[0])
                    if dst & data:
                        hits.append((func, i + 1, ln.strip(), t, waits))
                        break
            waits += 1
    return hits


def main(argv):
    total = 0
    for p in argv[1:]:
        for func, ln, st, vw, w in scan(p):
            total += 1
            print(f"{p}:{ln}: {func}: '{st}' then '{vw}' after {w} wait state(s)")
    print(f"{total} store-data hazard(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
