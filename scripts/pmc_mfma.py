"""MFMA utilisation and wave-state breakdown of the train step's conv kernels from the two PMC passes of
scripts/pmc_mfma.sh (verdict r3 item 3).

    python scripts/pmc_mfma.py gpurun_out/<TAG>_issue gpurun_out/<TAG>_lds [label] > profiles/<TAG>_mfma_busy.json

Units (calibrated here, not assumed): SQ_VALU_MFMA_BUSY_CYCLES advances 64 per v_mfma_f32_32x32x2_f32
(= its issue cycles on one SIMD; the conv family's per-step sum equals 64 x the valid-tap FLOPs / 4096
within 0.5 %), so MFMA utilisation = MFMA_BUSY / (dispatch duration x 2.4 GHz x 1,024 SIMDs).  No
measured-clock figure: GRBM_GUI_ACTIVE / 8 / duration reads high on dispatches shorter than ~0.3 ms
(MI355X_MICROARCH.md "DVFS give-back") and gave 2.3-6.7 GHz on these 5-60 us kernels,
so the utilisation is priced at the chip's maximum clock only (a lower bound on the in-kernel rate).
SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked at s_waitcnt / s_barrier) + SQ_WAIT_INST_ANY (issue-stalled: MFMA
pipe / dependency / LDS issue) + SQ_ACTIVE_INST_ANY (issuing); the fractions are of SQ_WAVE_CYCLES over
ALL waves of the kernel (loader waves included).  A step = the dispatches from one input gather to the next (else between consecutive k_adam
launches; the last complete step of the run is used (PMC serialises every dispatch)."""
import csv
import json
import os
import re
import sys
from collections import defaultdict

CONV = re.compile(r"k_(fwd|dgrad|wgrad|bwd)_(lds|x9)|k_(fwd_pair|bwd_quad)_(lds|x9)|k_conv_|k_stem_|k_reduce_slabs")
CLOCK_MAX_HZ = 2.4e9
SIMDS = 256 * 4


def load(d):
    rows, meta = defaultdict(dict), {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            i = int(r["Dispatch_Id"])
            rows[i][r["Counter_Name"]] = float(r["Counter_Value"])
            meta[i] = (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size"]),
                       int(r["Workgroup_Size"]), int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]),
                       int(r["LDS_Block_Size"]))
    return rows, meta


def last_step(meta):
    """The last complete step's dispatches.  Steps start at the bench's input gather (k_avmnist_gather, one
    per step) when the run has one — the AVMNIST step launches Adam more than once (per-encoder ranges) —
    else they end at each k_adam launch."""
    order = sorted(meta)
    if any("k_avmnist_gather" in meta[i][0] for i in order):
        steps, cur = [], None
        for i in order:
            if "k_avmnist_gather" in meta[i][0]:
                if cur:
                    steps.append(cur)
                cur = []
            if cur is not None:
                cur.append(i)
        return steps[-1], len(steps)  # the run's last segment (after the last gather) may be incomplete
    steps, cur, started = [], [], False
    for i in order:
        if started:
            cur.append(i)
        if "k_adam(" in meta[i][0]:
            if started and cur:
                steps.append(cur)
            cur, started = [], True
    return steps[-1], len(steps)


def short(name):
    m = re.search(r"(k_\w+(?:<[^()]*>)?)", name)
    return (m.group(1) if m else name[:60]).replace(" ", "")


def summarise(issue_dir, lds_dir):
    ri, mi = load(issue_dir)
    rl, ml = load(lds_dir)
    si, nsteps = last_step(mi)
    sl, _ = last_step(ml)
    lds_by_pos = {}
    if len(sl) == len(si):  # same dispatch sequence in both passes: pair them by position
        lds_by_pos = {a: b for a, b in zip(si, sl)}
    groups = defaultdict(lambda: defaultdict(float))
    fam = defaultdict(lambda: defaultdict(float))
    for i in si:
        name, t0, t1, grid, wg, vgpr, ldsb = mi[i]
        f = "conv" if CONV.search(name) else "bn" if "k_bn" in name else "adam" if "k_adam" in name else "other"
        key = (short(name), grid // max(wg, 1), wg, vgpr, ldsb) if f == "conv" else None
        c = dict(ri[i])
        c["dur_ns"] = t1 - t0
        c["launches"] = 1
        j = lds_by_pos.get(i)
        if j is not None:
            for k in ("SQ_INSTS_LDS", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                      "SQ_ACTIVE_INST_LDS"):
                c[k] = rl[j].get(k, 0.0)
            c["lds_pass_wave_cycles"] = rl[j].get("SQ_WAVE_CYCLES", 0.0)
        for k, v in c.items():
            fam[f][k] += v
            if key is not None:
                groups[key][k] += v

    def derive(c):
        dur = c["dur_ns"] * 1e-9
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        out = {"launches": int(c["launches"]), "device_us": round(c["dur_ns"] / 1e3, 2),
               "mfma_busy_cycles": busy, "mfma_count_f32_32x32x2": busy / 64,
               "mfma_util_at_2p4GHz": round(busy / (dur * CLOCK_MAX_HZ * SIMDS), 4) if dur else None,
               "wave_cycles": c.get("SQ_WAVE_CYCLES"),
               "frac_wait_any": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
               "frac_wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4),
               "frac_active_inst": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
               "waves": c.get("SQ_WAVES")}
        if "SQ_INSTS_LDS" in c:
            lwc = c.get("lds_pass_wave_cycles") or 1.0
            out.update({"lds_insts": c["SQ_INSTS_LDS"],
                        "frac_wait_inst_lds": round(c["SQ_WAIT_INST_LDS"] / lwc, 4),
                        "lds_bank_conflict_over_lds_active": round(c["SQ_LDS_BANK_CONFLICT"] /
                                                                   max(c["SQ_LDS_IDX_ACTIVE"], 1.0), 4)})
        return out

    res = {"families": {f: derive(c) for f, c in fam.items()}, "steps_in_run": nsteps,
           "paired_lds_pass": bool(lds_by_pos)}
    rows = []
    for (nm, wgs, wg, vgpr, ldsb), c in groups.items():
        d = derive(c)
        d.update({"kernel": nm, "workgroups": wgs, "wg_size": wg, "vgpr_agpr": vgpr, "lds_bytes": ldsb})
        rows.append(d)
    rows.sort(key=lambda d: -d["device_us"])
    res["conv_by_kernel_and_grid"] = rows
    return res


def main():
    issue_dir, lds_dir = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    out = {"what": __doc__.split("\n\n")[0], "label": label,
           "method": "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                     "SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE, and a second "
                     "pass SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE "
                     "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE, over `bench.py --steps 3 --warmup 2 "
                     "--no-cpu-baseline --profile-steps 0 --pcie-steps 0` (scripts/pmc_mfma.sh)",
           "units": "SQ_VALU_MFMA_BUSY_CYCLES = 64 per f32 32x32x2 MFMA (calibrated: conv family sum = 64 x "
                    "valid-tap FLOPs / 4096 within 0.5 %); wave-state fractions are of SQ_WAVE_CYCLES"}
    out.update(summarise(issue_dir, lds_dir))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
