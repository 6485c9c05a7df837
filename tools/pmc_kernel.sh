# HBM traffic of one kernel under a tool: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; one
# counter per pass), mean per dispatch of the kernels whose name contains <substr>, in MB
# (FETCH_SIZE doubled: the gfx950 16 B/lane correction of MI355X_MICROARCH.md, as bench.py does).
# usage: [env ...] bash tools/pmc_kernel.sh <tag> <tool.py under tools/> <kernel substring>
TAG=$1; TOOL=$2; SUB=$3
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/${TAG}_pmc_$c
  (cd tools && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d ../$d -o p -- python3 $TOOL > ../$d.log 2>&1) \
    || { tail -5 $d.log; exit 1; }
done
python3 - "$TAG" "$SUB" <<'PY'
import csv, glob, sys
tag, sub = sys.argv[1], sys.argv[2]
for c, mul in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
    f = glob.glob(f"gpurun_out/{tag}_pmc_{c}/**/*counter_collection.csv", recursive=True)
    rows = [r for r in csv.DictReader(open(f[0])) if sub in r["Kernel_Name"] and r["Counter_Name"] == c]
    v = [float(r["Counter_Value"]) * 1024 * mul / 1e6 for r in rows]
    print(f"{c}: {len(v)} dispatches of *{sub}*, mean {sum(v) / max(1, len(v)):.1f} MB per dispatch")
PY
