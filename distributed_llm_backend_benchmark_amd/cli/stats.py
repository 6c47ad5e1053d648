"""Offline statistics CLI (reference ``python stats.py`` with hand-edited INPUT_DIR/OUTPUT_DIR
constants, ``collectives/1d/stats.py:13-20``, ``collectives/3d/stats.py:16-30``)::

    python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 1d \
        --input-dir results/1d/rccl --output-dir stats/1d/rccl
    python -m distributed_llm_backend_benchmark_amd.cli.stats --mode 3d \
        --input-dir results/3d/rccl --output-dir stats/3d/rccl --impl rccl
"""

from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mode", choices=["1d", "3d"], required=True)
    ap.add_argument("--input-dir", required=True)
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--csv", default="benchmark_statistics.csv", help="1D CSV name")
    ap.add_argument("--impl", default="rccl", help="3D implementation label for CSV names")
    args = ap.parse_args(argv)
    from ..stats import stats1d, stats3d

    if args.mode == "1d":
        rows = stats1d.process_directory(args.input_dir, args.output_dir, args.csv)
        if rows:
            print(f"{'op':>14} {'P':>3} {'size':>7} {'p50 us':>10} {'busBW GB/s':>11}")
            for r in rows:
                bw = r.get("busbw_gbps")
                print(f"{r['operation']:>14} {r['num_ranks']:>3} {r['data_size_name']:>7} "
                      f"{r['median_time_us']:>10.2f} {bw if bw is None else round(bw, 2):>11}")
    else:
        rows = stats3d.process_directory(args.input_dir, args.output_dir, args.impl)
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main())
