"""ISA stats of the static 5v5 v7 rollout kernel (analysis aid; see isa_stats.sh)."""
import re, sys
lines = open(sys.argv[1]).read().split("\n")
name = sys.argv[2] if len(sys.argv) > 2 else "_ZN12_GLOBAL__N_117rollout_v2_kernelILi64ELb1ELi5ELi10EEEv10MlgEnvSpec"
st = next(i for i, l in enumerate(lines) if l.startswith(name) and ":" in l)
en = next(i for i in range(st, len(lines)) if lines[i].startswith("\t.size\t" + name))
k = lines[st:en]
meta = "\n".join(lines[st:en + 400])
def m(key):
    r = re.search(r"\.amdhsa_%s (\d+)" % key, meta)
    return r.group(1) if r else "?"
hdr = [i for i, l in enumerate(k) if "Loop Header: Depth=1" in l and "This Loop Header" in l]
bars = [i for i, l in enumerate(k) if l.strip() == "s_barrier"]
lo = hdr[-1] if hdr else 0
hi = max(b for b in bars if b > lo) if bars else len(k)
loop = [l.strip() for l in k[lo:hi + 1]]
ins = [l.split()[0] for l in loop if l and not l.startswith((";", ".")) and not l.endswith(":")]
cnt = lambda p: sum(1 for x in ins if x.startswith(p))
seg = [i for i, l in enumerate(loop) if l == "s_barrier"]
print("vgpr", m("next_free_vgpr"), "sgpr", m("next_free_sgpr"), "scratch", m("private_segment_fixed_size"),
      "| loop instrs", len(ins), "readlane", cnt("v_readlane"), "writelane", cnt("v_writelane"),
      "waitcnt", cnt("s_waitcnt"), "mfma", cnt("v_mfma"), "scratch_ops", cnt("scratch_") + cnt("buffer_"))
prev = 0
for j, b in enumerate(seg + [len(loop)]):
    part = [l.split()[0] for l in loop[prev:b] if l and not l.startswith((";", ".")) and not l.endswith(":")]
    print("  segment %d: %d instrs, readlane %d" % (j, len(part), sum(1 for x in part if x.startswith("v_readlane"))))
    prev = b
