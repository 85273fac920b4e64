"""Summarise rocprofv3 --pmc counter_collection CSVs: one row per dispatch of the kernels whose
name matches a pattern, with derived ratios (MFMA busy %, waves waiting %, LDS conflict rate).

usage: python tools/pmc_summary.py <pattern> <run_counter_collection.csv> [more.csv ...]
"""
import csv
import re
import sys
from collections import OrderedDict


def main():
    pat = re.compile(sys.argv[1])
    disp = OrderedDict()  # (file index, dispatch id) -> {counter: value}, name, grid, dur
    for fi, path in enumerate(sys.argv[2:]):
        with open(path) as f:
            for r in csv.DictReader(f):
                if not pat.search(r["Kernel_Name"]):
                    continue
                k = (fi, int(r["Dispatch_Id"]))
                d = disp.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])),
                                        "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                        "vgpr": r["VGPR_Count"], "lds": r["LDS_Block_Size"]})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for (fi, did), d in disp.items():
        name = re.sub(r"\(anonymous namespace\)::", "", d["name"])
        name = re.sub(r"\(.*", "", name)[:70]
        extra = []
        gui = d.get("GRBM_GUI_ACTIVE")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and gui:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy cycles over the 1024 SIMDs
            extra.append(f"mfma_busy {100 * d['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * 1024):5.1f}%")
        if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            extra.append(f"wait_any {100 * d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']:5.1f}%")
        if "SQ_WAIT_INST_ANY" in d and "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            extra.append(f"wait_inst {100 * d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES']:5.1f}%")
        if "SQ_ACTIVE_INST_VMEM" in d and "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            extra.append(f"vmem_active {100 * d['SQ_ACTIVE_INST_VMEM'] / d['SQ_WAVE_CYCLES']:5.1f}%")
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_ACTIVE_INST_LDS" in d and d["SQ_ACTIVE_INST_LDS"]:
            extra.append(f"lds_conflict {100 * d['SQ_LDS_BANK_CONFLICT'] / d['SQ_ACTIVE_INST_LDS']:5.1f}%")
        if "SQ_LEVEL_WAVES" in d and "SQ_WAVES" in d:
            pass
        if "TCC_HIT" in d and "TCC_MISS" in d and d["TCC_HIT"] + d["TCC_MISS"]:
            extra.append(f"L2hit {100 * d['TCC_HIT'] / (d['TCC_HIT'] + d['TCC_MISS']):5.1f}%")
        if "FETCH_SIZE" in d:
            extra.append(f"fetch {d['FETCH_SIZE'] / 1e3 * 2:8.1f} MB(x2)")
        if "WRITE_SIZE" in d:
            extra.append(f"write {d['WRITE_SIZE'] / 1e3:8.1f} MB")
        raw = " ".join(f"{k}={v:.3g}" for k, v in d.items() if k.isupper() or k[:2] in ("SQ", "TC", "TA", "GR"))
        print(f"[{fi}:{did:4d}] {d['us']:8.1f} us grid {d['grid']:6d} vgpr {d['vgpr']:>3s} lds {d['lds']:>6s} {name}")
        print("      " + "  ".join(extra))
        print("      " + raw)


if __name__ == "__main__":
    main()
