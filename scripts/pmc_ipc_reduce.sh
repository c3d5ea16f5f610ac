#!/bin/bash
# Raw TCC/EA request counters of the exact ipc round's reduce role
# (bench/ipc_reduce_role.py: one process, pre-set flags), one rocprofv3 pass
# per counter group, then bytes per dispatch: read should be N x block, write
# 2 x block (output + reduced row).  Summary: gpurun_out/pmc_ipc/summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/${PMC_OUT:-pmc_ipc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench/ipc_reduce_role.py ${PMC_BENCH_ARGS:---n 2,8 --block-mb 32 --threads 256 --modes sys,plain} --iters 3"
i=0
for C in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p$i -o run -- python3 $ARGS > $O/p$i.log 2>&1 || { echo "pass $i ($C) rc=$?"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O/p1 $O/p2 > $O/summary.txt <<'PY'
import collections, csv, glob, os, sys
def load(d):
    disp = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "ipc_reduce_kernel" not in r.get("Kernel_Name", ""):
                continue
            e = disp.setdefault(int(r["Dispatch_Id"]), [int(r["Grid_Size"]), {}, 0])
            e[1][r["Counter_Name"]] = float(r["Counter_Value"])
            e[2] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return [disp[k] for k in sorted(disp)]
p1, p2 = load(sys.argv[1]), load(sys.argv[2])
print("dispatch  grid   RD_MiB  WR_MiB  DRAM%   us")
for i, (a, b) in enumerate(zip(p1, p2)):
    c = dict(a[1]); c.update(b[1])
    rd = 128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0)
    wr = 64 * c.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (c.get("TCC_EA0_WRREQ_sum", 0) - c.get("TCC_EA0_WRREQ_64B_sum", 0))
    dram = 100 * c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / max(1, c.get("TCC_EA0_RDREQ_sum", 1))
    print(f"{i:8d} {a[0]:6d} {rd/2**20:8.1f} {wr/2**20:7.1f} {dram:6.1f} {a[2]/1e3:7.1f}")
PY
cat $O/summary.txt
