"""Per-step HBM traffic by kernel family from the two PMC passes of scripts/pmc_traffic.sh.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/<ver>_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  Per MI355X_MICROARCH.md
("HBM"), gfx950's FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced read —
the load shape of every hot kernel here (global_load_lds_dwordx4 / dwordx4) — so fetched bytes are
2 × FETCH_SIZE; WRITE_SIZE is exact for 16-B stores.  A "step" is the dispatches between two
consecutive k_adam launches (the optimizer closes every step); the steady-state figure is the
median over the complete steps of the run.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

FAMILIES = [("conv", ("k_fwd_lds", "k_fwd_pair_lds", "k_dgrad_lds", "k_wgrad_lds", "k_bwd_lds", "k_bwd_quad_lds", "k_fwd_x9", "k_fwd_pair_x9", "k_dgrad_x9", "k_wgrad_x9", "k_bwd_x9", "k_bwd_quad_x9", "k_conv_", "k_stem_", "k_reduce_slabs")),
            ("bn", ("k_bn_", "k_bn1d")), ("pool", ("k_maxpool", "k_avgpool")), ("adam", ("k_adam",)),
            ("gather", ("k_avmnist_gather",)), ("head", ("k_head_", "k_gemm_small", "k_gemm_pair", "k_splitk_reduce",
                                                         "k_cross_entropy", "k_act_bwd", "k_dropout")),
            ("mmimdb_ew", ("k_gmu", "k_maxout", "k_bce")),
            ("mosi", ("k_lstm_", "k_textcnn", "k_seq_gather", "k_sumsq", "k_clip_coef"))]  # "head" = every small-GEMM (Linear) launch


def family(name: str) -> str:
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return "other"


def load(d: str, counter: str):
    rows = []
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    return rows


def steps(rows):
    """Complete steps: from one input gather (k_avmnist_gather, one per bench step) to the next when the run
    has them — the AVMNIST step launches Adam more than once (per-encoder ranges) — else the dispatches
    between consecutive k_adam launches."""
    if any("k_avmnist_gather" in name for _, name, _ in rows):
        out, cur = [], None
        for _, name, v in rows:
            if "k_avmnist_gather" in name:
                if cur:
                    out.append(cur)
                cur = []
            if cur is not None:
                cur.append((name, v))
        return out
    out, cur, started = [], [], False
    for _, name, v in rows:
        if started:
            cur.append((name, v))
        if "k_adam(" in name:
            if started and cur:
                out.append(cur)
            cur, started = [], True
    return out


def per_step(rows, scale):
    res = []
    for st in steps(rows):
        fam = defaultdict(float)
        n = defaultdict(int)
        for name, v in st:
            f = family(name)
            fam[f] += v * scale
            n[f] += 1
        res.append((dict(fam), dict(n)))
    return res


def main(fetch_dir: str, write_dir: str) -> None:
    rd = per_step(load(fetch_dir, "FETCH_SIZE"), 2.0)
    wr = per_step(load(write_dir, "WRITE_SIZE"), 1.0)
    fams = sorted({f for s, _ in rd + wr for f in s})
    bench_args = sys.argv[3] if len(sys.argv) > 3 else "--steps 3 --warmup 2 --no-cpu-baseline"
    out = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     f"`bench.py {bench_args}`; read bytes = 2 x FETCH_SIZE "
                     "(gfx950 wide-read correction), write bytes = WRITE_SIZE; per step = dispatches "
                     "from one input gather to the next (else between consecutive k_adam launches); median "
                     "over complete steps",
           "steps_read_pass": len(rd), "steps_write_pass": len(wr), "per_step_bytes": {}}
    for f in fams:
        r = statistics.median([s.get(f, 0.0) for s, _ in rd]) if rd else None
        w = statistics.median([s.get(f, 0.0) for s, _ in wr]) if wr else None
        launches = statistics.median([n.get(f, 0) for _, n in rd]) if rd else None
        out["per_step_bytes"][f] = {"read": r, "write": w, "total": (r or 0) + (w or 0), "launches": launches}
    out["per_step_total_bytes"] = sum(v["total"] for v in out["per_step_bytes"].values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
