"""Scan the built codec's gfx950 machine code for the store-data hazard behind round 5's
r5m wrong stores.

A 12/16-byte vector store must read its data registers before the next VALU instruction
may overwrite them (one wait state).  The compiler inserts that wait state for buffer
stores whose soffset is a constant, but NOT for a buffer store whose soffset is an SGPR
(the ISA manuals exempt that form), and on gfx950 such a store has been seen to write the
overwritten values: the r5m build of the sign receive stored wrong x / memory values at
~0.1 % of the elements while x_hat and the packed words were right.
The codec therefore never gives a 12/16-byte store an SGPR soffset; this scan checks the
shipped library for (a) any such store and (b) any 12/16-byte store directly followed by a
VALU that overwrites one of its data registers.

    python tools/isa_hazards.py [path/to/libchoco_codec.so]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
_WIDE_STORE = re.compile(r"(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b")


def _regs(tok):
    m = re.match(r"[va]\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"[va](\d+)$", tok)
    return {int(m.group(1))} if m else set()


def disassemble(lib):
    """The disassembly of every gfx950 code object bundled in `lib` (one string each)."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, os.path.basename(lib))
        shutil.copy(lib, src)
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "--offloading", src], cwd=td, check=True,
                       capture_output=True)
        for f in sorted(os.listdir(td)):
            if f.endswith("gfx950"):
                r = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--mcpu=gfx950",
                                    os.path.join(td, f)], check=True, capture_output=True, text=True)
                out.append(r.stdout)
    return out


def scan_text(text):
    """(wide stores, those with an SGPR soffset, [(store, next instruction)] hazards)."""
    insts = []
    for ln in text.splitlines():
        t = ln.split("//")[0].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("Disassembly"):
            continue
        insts.append(t)
    n_wide = n_sreg = 0
    bad = []
    for i, t in enumerate(insts):
        if not _WIDE_STORE.match(t):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        data = _regs(ops[1] if t.startswith(("global", "flat", "scratch")) else ops[0])
        n_wide += 1
        if t.startswith("buffer") and len(ops) > 3 and re.match(r"s\d", ops[3].split()[0]):
            n_sreg += 1
        nxt = insts[i + 1] if i + 1 < len(insts) else ""
        if nxt.startswith("v_") and " " in nxt:
            dst = nxt.split(None, 1)[1].split(",")[0].strip()
            if _regs(dst) & data:
                bad.append((t, nxt))
    return n_wide, n_sreg, bad


def scan_library(lib):
    n_wide = n_sreg = 0
    bad = []
    for text in disassemble(lib):
        a, b, c = scan_text(text)
        n_wide, n_sreg, bad = n_wide + a, n_sreg + b, bad + c
    return n_wide, n_sreg, bad


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "chocosgd_amd", "lib", "libchoco_codec.so")
    n_wide, n_sreg, bad = scan_library(lib)
    print(f"{lib}: {n_wide} stores of 12/16 B, {n_sreg} with an SGPR soffset, "
          f"{len(bad)} followed at once by a VALU overwriting their data")
    for s, v in bad[:10]:
        print("   ", s, "=>", v)
    sys.exit(1 if (n_sreg or bad) else 0)
