"""Markdown rows for DESIGN.md §4 "End-to-end training, round 4" from the two accuracy-protocol summaries.

    python scripts/acc_design_table.py profiles/r4_accuracy_parity.json profiles/r4_accuracy_parity_pretrained.json
"""
import json
import math
import sys


def needed(sd, mean, margin=0.2, t=1.7):
    room = margin - abs(mean)
    return None if room <= 0 else math.ceil((t * sd / room) ** 2)


def main():
    print("| setting (paired runs) | end point | reference | ours | delta (pp) | TOST 90 % CI (pp) | paired sd (pp) "
          "| runs needed |")
    print("|---|---|---|---|---|---|---|---|")
    for path in sys.argv[1:]:
        d = json.load(open(path))
        for key, label in (("test_accuracy_ai", "**test accuracy of best.pth, pattern ai (pre-registered)**"),
                           ("test_accuracy_all", "test accuracy of best.pth, patterns ai / a / i")):
            x = d[key]
            p = x["paired"]
            eq = "equivalent" if p["equivalent_at_0.2pp"] else "not equivalent"
            n = needed(p["paired_sd_pp"], p["delta_pp"])
            print(f"| {d['setting']} ({d['paired_runs']}) | {label} | {100 * x['reference_mean']:.2f} % | "
                  f"{100 * x['ours_mean']:.2f} % | {p['delta_pp']:+.3f} | [{p['ci90_pp'][0]:+.3f}, {p['ci90_pp'][1]:+.3f}] "
                  f"{eq} | {p['paired_sd_pp']:.2f} | {n if n is not None else '—'} |")


if __name__ == "__main__":
    main()
