"""Per-kernel FP64-pipe breakdown from rocprofv3 --pmc passes (tools/pmc_run.sh with PMC_GROUPS covering
SQ_INSTS_VALU / SQ_INSTS_MFMA / SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE / the F64 VALU classes).

gfx950: FP64 MFMA and FP64 VALU share one pipe (SQ_VALU_MFMA_COEXEC_CYCLES reads 0), so the kernel's pipe
occupancy per SIMD is the MFMA-busy fraction plus the VALU-issue fraction:
  mfma  = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)
  valu  = 4 cycles × (SQ_INSTS_VALU − SQ_INSTS_MFMA) / 1024 / (GRBM_GUI_ACTIVE / 8)   (wave64 on a 16-lane SIMD)
Usage: python tools/pmc_pipe.py gpurun_out/<dir> [more dirs] > profiles/<name>.json
       python tools/pmc_pipe.py --table gpurun_out/<dir>   (one text line per kernel, every kernel of the run)
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    vals = collections.defaultdict(list)
    for path in sorted(glob.glob(os.path.join(d, "pass*_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            vals[(r["Kernel_Name"].split("(")[0].strip(), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def table(d):
    m = load(d)
    print(f"# {d}: per kernel (averaged over its dispatches) — XCD cycles = GRBM_GUI_ACTIVE / 8; FP64 pipe = MFMA busy + "
          "VALU issue per SIMD; wait = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES; L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS); "
          "FETCH_SIZE / WRITE_SIZE in MB as counted (gfx950: fabric bytes = 2 x FETCH_SIZE)")
    for kern in sorted({k for k, _ in m}):
        c = {name: v for (k, name), v in m.items() if k == kern}
        gui = c.get("GRBM_GUI_ACTIVE")
        if not gui:
            continue
        cyc = gui / 8
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / cyc
        va = 4 * (c.get("SQ_INSTS_VALU", 0.0) - c.get("SQ_INSTS_MFMA", 0.0)) / 1024 / cyc
        wc = max(c.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        h, mi = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        print(f"{kern[:64]:64s} cycles {cyc:9.0f}  mfma {mf:5.3f}  valu {va:5.3f}  wait {c.get('SQ_WAIT_INST_ANY', 0.0) / wc:4.2f}"
              f"  L2 hit {h / max(h + mi, 1.0):5.3f}  fetch {c.get('FETCH_SIZE', 0.0) / 1024:7.1f}  write {c.get('WRITE_SIZE', 0.0) / 1024:6.1f}")


def main():
    if sys.argv[1] == "--table":
        for d in sys.argv[2:]:
            table(d)
        return
    out = {}
    for d in sys.argv[1:]:
        m = load(d)
        for kern in sorted({k for k, _ in m}):
            if "posterior" not in kern and "kernel_block" not in kern:
                continue
            c = {name: v for (k, name), v in m.items() if k == kern}
            gui = c.get("GRBM_GUI_ACTIVE")
            e = {"counters": c, "source": d}
            if gui:
                cyc = gui / 8
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc
                if "SQ_INSTS_VALU" in c and "SQ_INSTS_MFMA" in c:
                    e["valu_issue_frac"] = 4 * (c["SQ_INSTS_VALU"] - c["SQ_INSTS_MFMA"]) / 1024 / cyc
                if "mfma_busy_frac" in e and "valu_issue_frac" in e:
                    e["fp64_pipe_busy_frac"] = e["mfma_busy_frac"] + e["valu_issue_frac"]
            f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                               "SQ_INSTS_VALU_TRANS_F64"))
            if f64:
                e["fp64_valu_insts"] = f64
            if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
                e["hbm_bytes"] = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024
            if "TCC_HIT_sum" in c:
                h, mi = c["TCC_HIT_sum"], c.get("TCC_MISS_sum", 0.0)
                e["l2_hit_rate"] = h / (h + mi) if h + mi else None
            out[f"{os.path.basename(d.rstrip('/'))}:{kern}"] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
