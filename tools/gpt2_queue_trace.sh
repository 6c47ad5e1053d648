#!/bin/bash
# One GPT-2 DDP world-1 run under rocprofv3 kernel + HIP runtime trace:
# every dispatch's hardware queue (Queue_Id) and stream (Stream_Id), every stream-creating HIP
# call, and the run's own role -> hipStream_t map (result JSON "streams"). Keeps the kernel trace
# (gzip) and only the stream-related HIP API rows. Usage on the box: bash tools/gpt2_queue_trace.sh OUT
set -eu
O=$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
  -d "$GRAFT_REPO_ROOT/$O/raw" -o gpt2 -- \
  python3 -m distributed_llm_backend_benchmark_amd.cli.train_ddp --steps 10 --warmup 6 \
  --output "$GRAFT_REPO_ROOT/$O/gpt2_traced.json"
cd "$GRAFT_REPO_ROOT"
python3 - "$O" <<'EOF'
import csv, glob, gzip, os, shutil, sys
o = sys.argv[1]
kt = glob.glob(f"{o}/raw/**/*kernel_trace.csv", recursive=True)
ht = glob.glob(f"{o}/raw/**/*hip_api_trace.csv", recursive=True)
for f in kt:
    with open(f, "rb") as a, gzip.open(f"{o}/kernel_trace.csv.gz", "wb") as b:
        shutil.copyfileobj(a, b)
for f in ht:
    with open(f) as a, open(f"{o}/hip_stream_calls.csv", "w", newline="") as b:
        r = csv.DictReader(a)
        w = csv.DictWriter(b, fieldnames=r.fieldnames)
        w.writeheader()
        for row in r:
            if "Stream" in row.get("Function", "") and "Synchronize" not in row["Function"] \
                    and "Query" not in row["Function"] and "WaitEvent" not in row["Function"]:
                w.writerow(row)
shutil.rmtree(f"{o}/raw")
print("kept", kt, ht)
EOF
