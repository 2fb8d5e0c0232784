#!/bin/bash
# GPU box: k_dns_parse alone -- timing, then SQ counter passes (tools/pmc_sq.sh with tools/dns_only.py).
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
timeout -k 10 120 python tools/dns_only.py || exit 1
cd /tmp
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_CYCLES SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS"; do
  i=$((i+1)); TAG=dsq$i; rm -rf $R/gpurun_out/pmc/$TAG
  REPS=2 timeout -s KILL 90 rocprofv3 --pmc $PMC -d $R/gpurun_out/pmc/$TAG -o run -- python3 $R/tools/dns_only.py > $R/gpurun_out/pmc/$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i rc=$rc"; tail -5 $R/gpurun_out/pmc/$TAG.log; exit 1; }
done
python3 - "$R/gpurun_out/pmc" <<'PY'
import collections, glob, sqlite3, statistics, sys
acc = collections.defaultdict(list)
for d in sorted(glob.glob(sys.argv[1] + "/dsq*")):
    for db in glob.glob(d + "/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            if "k_dns_parse" in k:
                acc[cn].append(v)
for cn, v in sorted(acc.items()):
    print("%-28s n=%3d median=%.6g" % (cn, len(v), statistics.median(v)))
PY
