#!/usr/bin/env python3
"""Disassemble the gfx950 code object already inside the built library (no recompilation):
python tools/isa_dump.py [kernel-substring ...] [-loops] [-v]

Finds the clang offload bundle in libfhespear_hip.so (.hip_fatbin), extracts the
amdgcn-amd-amdhsa--gfx950 ELF, runs llvm-objdump -d, and prints per-kernel instruction counts (and,
with -loops, per basic block VALU counts) like tools/isa_stats.py does from a fresh -S compile."""
import collections
import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("FHS_ISA_LIB") or os.path.join(ROOT, "fhe-spear_amd", "lib", "libfhespear_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_object(lib=LIB):
    data = open(lib, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        off = pos + len(MAGIC) + 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if "gfx950" in triple:
                return data[pos + o:pos + o + sz]
        pos = data.find(MAGIC, pos + 1)
    raise SystemExit("no gfx950 code object found")


def disasm():
    co = "/tmp/fhs_gfx950.co"
    open(co, "wb").write(code_object())
    return subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", co], capture_output=True,
                          text=True, check=True).stdout


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("-")] or ["k_modup_h"]
    text = disasm()
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", text)
    for f in funcs:
        m = re.match(r"[0-9a-f]+ <(\S+)>:", f)
        if not m or not any(n in m.group(1) for n in names):
            continue
        lines = [l.strip() for l in f.splitlines()[1:] if l.strip() and not l.strip().startswith(";")]
        ins = [l.split()[0] for l in lines]
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{m.group(1)[:80]}: instr {len(ins)} valu {valu} mad64 {c['v_mad_u64_u32']} "
              f"vmem {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))} "
              f"lds {sum(v for k, v in c.items() if k.startswith('ds_'))} gpridx {c['s_set_gpr_idx_on']} "
              f"readfirstlane {c['v_readfirstlane_b32']}")
        if "-v" in sys.argv:
            print("   ", c.most_common(40))


if __name__ == "__main__":
    main()
