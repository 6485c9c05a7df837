# SQ counters of one kernel under a tool (one rocprofv3 --pmc pass, <= 8 SQ counters), mean per
# dispatch of the kernels whose name contains <substr>.
# usage: [env ...] bash tools/pmc_sq.sh <tag> <tool.py under tools/> <kernel substring> [counters...]
TAG=$1; TOOL=$2; SUB=$3; shift 3
CTRS=${*:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
d=gpurun_out/${TAG}_sq
(cd tools && timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d ../$d -o p -- python3 $TOOL > ../$d.log 2>&1) \
  || { tail -5 $d.log; exit 1; }
python3 - "$d" "$SUB" <<'PY'
import csv, glob, sys, collections
d, sub = sys.argv[1], sys.argv[2]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if sub in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:28s} {len(v):4d} dispatches  mean {sum(v) / len(v):14.4g}")
PY
