"""Per-launch counter summary of the rollout kernels from scripts/gpu_counters.sh passes -> profiles/counters.json.

* hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B): on gfx950 FETCH_SIZE reports half the bytes of wide
  coalesced reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B-per-lane stores.
* mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): MFMA-busy cycles (summed over every
  SIMD) over the SIMD-cycles of the dispatch (GRBM_GUI_ACTIVE is summed over the 8 XCDs).
* wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier), wait_inst_frac likewise,
  lds_conflict_per_lds_inst = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS, valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA.
Averages over the profiled launches of each kernel (every launch of a name has the same shape)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, commit = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "unknown")
# the rollout kernels and the learners' kernels (QMIX learner.hip, REFIL refil_learner.hip, shared wgrad)
FILT = tuple(os.environ.get("MLG_CNT_FILTER", "rollout,agent_,rec4_mixpre,mix_td,wgrad_block,finish_kernel,prep_kernel,"
                            "hyper_fwd,hyper_bwd,ent_fwd,ent_bwd,rec_kernel,rec4_kernel,rec_bwd,q_kernel,prologue_kernel,bwd4_wgrad").split(","))


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch] (per pass for GRBM)
for f in glob.glob(os.path.join(root, "*", "*", "**", "*counter_collection.csv"), recursive=True):
    pass_name = f.split(os.sep)[len(root.rstrip(os.sep).split(os.sep)) + 1]
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if not any(x in k for x in FILT):
            continue
        c = r["Counter_Name"]
        key = c if c != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE@{pass_name}"
        per[(short(k), key, r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, _), v in per.items():
        vals[k][c].append(v)
out = {}
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    d = {"commit": commit, "dispatches": max(len(v) for v in cs.values()), "raw": m}
    if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
        d["fetch_kb_raw"], d["write_kb"] = m.get("FETCH_SIZE"), m.get("WRITE_SIZE")
        d["hbm_bytes_per_launch"] = (2 * m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) * 1024.0
    g2 = m.get("GRBM_GUI_ACTIVE@sq2")
    if g2 and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        d["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * g2 / 8.0)
        d["kernel_cycles"] = g2 / 8.0
    if "SQ_WAVE_CYCLES" in m:
        d["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
        d["wait_inst_frac"] = m.get("SQ_WAIT_INST_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
        d["active_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
    if m.get("SQ_INSTS_LDS"):
        d["lds_conflict_per_lds_inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
    if m.get("SQ_INSTS_MFMA"):
        d["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_INSTS_MFMA"]
    out[k] = d
# annotations that are not counters (bench.py's latency floor reads them): kept when a kernel is re-collected
KEEP = ("one_env_step_cycles", "one_env_step_source", "one_env_step_commit")
if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):  # merge into an existing counters.json (other kernels kept)
    prev = json.load(open(sys.argv[3])).get("kernels", {})
    for k, d in out.items():
        d.update({a: prev[k][a] for a in KEEP if a in prev.get(k, {}) and a not in d})
    prev.update(out)
    out = prev
print(json.dumps({"kernels": out, "note": __doc__.strip().splitlines()[0]}, indent=1))
