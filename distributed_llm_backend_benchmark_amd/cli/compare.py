"""Compare our collective statistics with the reference's published CSVs.

    python -m distributed_llm_backend_benchmark_amd.cli.compare --mode 1d \
        --ours results/r01_world1/stats/1d/rccl/benchmark_statistics_ext.csv \
        --ref /root/reference/collectives/1d/stats/*/benchmark_statistics.csv \
        --any-ranks --output results/compare_1d.csv

``--ref`` takes several CSVs (one per reference implementation); the best reference p50 per
configuration is used. ``--any-ranks`` pairs our rows with reference rows of any rank count
(e.g. world-1 measurements against the reference's P=2..16). Prints a markdown table.
"""

from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mode", choices=["1d", "3d"], required=True)
    ap.add_argument("--ours", nargs="+", required=True, help="our stats CSV(s)")
    ap.add_argument("--ref", nargs="+", required=True, help="reference stats CSV(s)")
    ap.add_argument("--any-ranks", action="store_true")
    ap.add_argument("--ops", default=None, help="comma list filter")
    ap.add_argument("--output", default=None, help="write the joined table as CSV")
    args = ap.parse_args(argv)
    from ..stats import compare as C

    load = C.load_1d if args.mode == "1d" else C.load_3d
    ours, ref = load(args.ours), load(args.ref)
    rows = C.compare(ours, ref, match_ranks=not args.any_ranks)
    if args.ops:
        keep = set(args.ops.split(","))
        rows = [r for r in rows if r["operation"] in keep]
    if args.output:
        C.write_csv(rows, args.output)
    print(C.markdown(rows))
    print(f"{len(rows)} configurations compared", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
