"""Instruction mix of the kernels in a device asm file whose symbol contains a pattern (analysis aid).
usage: isa_mix.py file.s pattern"""
import re
import sys
from collections import Counter

L = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
for st, l in enumerate(L):
    m = re.match(r"^(_Z\S*):", l)
    if not m or pat not in m.group(1):
        continue
    name = m.group(1)
    en = next(i for i in range(st, len(L)) if L[i].startswith("\t.size\t" + name))
    ins = [x.strip().split()[0] for x in L[st + 1:en] if x.strip() and not x.strip().startswith((";", ".")) and not x.strip().endswith(":")]
    c = Counter(ins)
    meta = "\n".join(L[st:en + 400])
    g = lambda key: (re.search(r"\.amdhsa_%s (\d+)" % key, meta) or [None, "?"])[1]
    print(name[:70], "vgpr", g("next_free_vgpr"), "accum_offset", g("accum_offset"), "sgpr", g("next_free_sgpr"),
          "scratch", g("private_segment_fixed_size"), "instrs", len(ins))
    for p in ["v_pk_fma_f32", "v_fma_f32", "v_fmac_f32", "v_mfma", "v_exp_f32", "ds_read_b128", "ds_read", "ds_write",
              "v_readlane", "v_writelane", "v_accvgpr", "buffer_load", "global_load", "scratch_", "_dpp", "v_pk_mul_f32",
              "v_pk_add_f32", "s_waitcnt", "v_cndmask", "v_perm", "v_and", "v_lshl", "v_add"]:
        print("   %-14s %d" % (p, sum(v for kk, v in c.items() if kk.startswith(p) or (p.startswith("_") and p in kk))))
