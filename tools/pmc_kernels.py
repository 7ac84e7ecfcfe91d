"""Summary of tools/pmc_kernels.sh: per kernel (mean over dispatches) the issue / wait split
and unit busy fractions.  python tools/pmc_kernels.py gpurun_out/TAG

SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles summed over waves
(MI355X_MICROARCH.md constants table); SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over
SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Printed as fractions of wave cycles
(issue/wait) and of SIMD cycles (MFMA busy = MFMA_BUSY / (GUI_ACTIVE/8 * 1024 SIMDs)), TD/TA
busy per CU cycle (TD_TD_BUSY_sum / (GUI_ACTIVE/8 * 256))."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), short(r["Kernel_Name"]))
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (_, k), cs in per.items():
            for c, v in cs.items():
                acc[k][c].append(v)
    return acc


def main():
    d = sys.argv[1]
    data = defaultdict(dict)
    for p in ("pa", "pb", "pc"):
        for k, cs in load(os.path.join(d, p)).items():
            for c, vs in cs.items():
                data[k][c + ("" if c != "GRBM_GUI_ACTIVE" else "@" + p)] = sum(vs) / len(vs)
    rows = []
    for k, c in data.items():
        g = c.get("GRBM_GUI_ACTIVE@pa") or c.get("GRBM_GUI_ACTIVE@pb")
        if not g or "SQ_WAVE_CYCLES" not in c:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        clk = g / 8.0
        f = lambda n, base=wc: c.get(n, float("nan")) / base if base else float("nan")  # noqa: E731
        gb = c.get("GRBM_GUI_ACTIVE@pb", g) / 8.0
        gc = c.get("GRBM_GUI_ACTIVE@pc", g) / 8.0
        rows.append((clk, k, {
            "clk": clk,
            "wait_any": f("SQ_WAIT_ANY"), "wait_inst": f("SQ_WAIT_INST_ANY"), "act_any": f("SQ_ACTIVE_INST_ANY"),
            "act_valu": f("SQ_ACTIVE_INST_VALU"), "act_lds": f("SQ_ACTIVE_INST_LDS"), "act_vmem": f("SQ_ACTIVE_INST_VMEM"),
            "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (gb * 1024),
            "coexec": c.get("SQ_VALU_MFMA_COEXEC_CYCLES", float("nan")) / (gb * 1024),
            "valu/mfma": c.get("SQ_INSTS_VALU", float("nan")) / max(c.get("SQ_INSTS_MFMA", 0.0), 1.0),
            "lds/mfma": c.get("SQ_INSTS_LDS", float("nan")) / max(c.get("SQ_INSTS_MFMA", 0.0), 1.0),
            "salu/mfma": c.get("SQ_INSTS_SALU", float("nan")) / max(c.get("SQ_INSTS_MFMA", 0.0), 1.0),
            "td_busy": c.get("TD_TD_BUSY_sum", float("nan")) / (gc * 256),
            "ta_busy": c.get("TA_TA_BUSY_sum", float("nan")) / (gc * 256),
            "lds_conf": c.get("SQ_LDS_BANK_CONFLICT", float("nan")) / max(c.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0),
            "waves": c.get("SQ_WAVES", float("nan")),
        }))
    rows.sort(key=lambda r: -r[0])
    keys = ["clk", "wait_any", "wait_inst", "act_any", "act_valu", "act_lds", "act_vmem", "mfma_busy", "coexec",
            "valu/mfma", "lds/mfma", "salu/mfma", "td_busy", "ta_busy", "lds_conf", "waves"]
    print("| kernel | " + " | ".join(keys) + " |")
    print("|---|" + "---|" * len(keys))
    for _, k, v in rows[:30]:
        print(f"| `{k}` | " + " | ".join(f"{v[x]:.3g}" for x in keys) + " |")


if __name__ == "__main__":
    main()
