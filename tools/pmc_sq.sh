#!/bin/bash
# GPU box: SQ instruction / cycle counters of the headline bench kernel, one rocprofv3 --pmc pass
# per counter group (never combined with tracing domains), summarised per kernel via sqlite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
ARGS=${ARGS:---steps 64 --warmup 8 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch}
i=0
KFILT=${KFILT:-k_parse_seg}
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_CYCLES" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_BUSY_CU_CYCLES"; do
  i=$((i+1)); TAG=sq$i; rm -rf $R/gpurun_out/pmc/$TAG
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc $PMC -d $R/gpurun_out/pmc/$TAG -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -5 $R/gpurun_out/pmc/$TAG.log; exit 1; }
done
KFILT=$KFILT python3 - "$R/gpurun_out/pmc" <<'PY'
import collections, glob, os, sqlite3, statistics, sys
acc = collections.defaultdict(list)
for d in sorted(glob.glob(sys.argv[1] + "/sq*")):
    dbs = glob.glob(d + "/**/*.db", recursive=True)
    if not dbs:
        continue
    c = sqlite3.connect(dbs[0])
    for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        if os.environ.get("KFILT", "k_parse_seg") in k:
            acc[(k[:50], cn)].append(v)
for (k, cn), v in sorted(acc.items()):
    print("%-50s %-28s n=%4d median=%.6g" % (k, cn, len(v), statistics.median(v)))
PY
