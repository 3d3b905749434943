"""Static ISA statistics of selected kernels: python tools/isa_stats.py [kernel-substring ...]
Compiles fhe-spear_amd/csrc/fhs_kernels.hip to gfx950 assembly and reports VGPRs, scratch and
per-opcode counts for each matching kernel (a quick check of instruction count per butterfly)."""
import collections, re, subprocess, sys, os
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "fhe-spear_amd", "csrc", "fhs_kernels.hip")
out = "/tmp/fhs_kernels_isa.s"
defs = [a for a in sys.argv[1:] if a.startswith("-D")]
names = [a for a in sys.argv[1:] if not a.startswith("-D")] or ["k_ntt_fwdILi14"]
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                src, "-o", out] + defs, check=True, stderr=subprocess.DEVNULL)
s = open(out).read()
for name in names:
    for m in re.finditer(r"^(_Z\S*%s\S*):" % re.escape(name), s, re.M):
        sym = m.group(1)
        j = s.find("s_endpgm", m.end())
        ins = [l.strip().split()[0] for l in s[m.end():j].splitlines()
               if l.strip() and not l.strip().startswith((".", ";"))]
        meta = s[s.find(".amdhsa_kernel " + sym):][:4000]
        vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta)
        sc = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta)
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{sym[:70]}: vgpr {vg and vg.group(1)} scratch {sc and sc.group(1)} instr {len(ins)} valu {valu} "
              f"nop {c['s_nop']} mov {c['v_mov_b32_e32']} vmem {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))} "
              f"smem {sum(v for k, v in c.items() if k.startswith('s_load'))} lds {sum(v for k, v in c.items() if k.startswith('ds_'))}")
        if "-v" in sys.argv:
            print("   ", c.most_common(30))

if "-loops" in sys.argv:
    for name in names:
        for m in re.finditer(r"^(_Z\S*%s\S*):" % re.escape(name), s, re.M):
            j = s.find("s_endpgm", m.end())
            body = s[m.end():j].splitlines()
            labels = [(i, l) for i, l in enumerate(body) if l.startswith(".LBB")] + [(len(body), "end")]
            for (i, l), (i2, _) in zip(labels, labels[1:]):
                seg = [x.strip().split()[0] for x in body[i + 1:i2] if x.strip() and not x.strip().startswith((".", ";"))]
                c = collections.Counter(seg)
                v = sum(n for k, n in c.items() if k.startswith("v_"))
                if v >= 20:
                    print(f"  {l.split()[0]:12s} valu {v:4d} mad64 {c['v_mad_u64_u32']:3d} mov {c['v_mov_b32_e32']:3d} "
                          f"lds {sum(n for k, n in c.items() if k.startswith('ds_'))} vmem {sum(n for k, n in c.items() if k.startswith('global_'))} {l[l.find(';'):][:40] if ';' in l else ''}")
