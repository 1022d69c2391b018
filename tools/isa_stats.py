"""Instruction-class counts of the fused kernels in a gfx950 assembly listing (static counts):
  hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S crdt-enc_amd/csrc/ce_fused.hip -o fused.s
  python3 tools/isa_stats.py fused.s"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_ZN2ce\d+k_open_fold\w+):", s, re.M):
    name = m.group(1)
    body = s[m.end(): s.index(".Lfunc_end", m.end())].split("\n")
    ins = [l.split(";")[0].strip() for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    ins = [l for l in ins if l]
    ops = [l.split()[0] for l in ins]
    c = lambda p: sum(1 for o in ops if o.startswith(p))
    print("%-44s total %5d valu %5d mad64 %4d gload %3d ds %4d scratch %3d waitcnt %4d cbranch %3d sched %s" % (
        name[8:52], len(ops), c("v_"), c("v_mad_u64_u32"), c("global_load"), c("ds_"), c("scratch_"),
        c("s_waitcnt"), c("s_cbranch"), ""))
