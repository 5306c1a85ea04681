#!/bin/bash
# Counters for the balanced wire kernel on packed IMIX (tools/lb_ab.py workloads), one pass each.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_lb
mkdir -p $O
timeout -k 10 120 ./tests/c/abi_smoke --gpu > $O/abi_smoke.log 2>&1
P="python3 tools/lb_ab.py"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/a -o p -- $P > $O/a.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- $P > $O/b.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $P > $O/kt.log 2>&1
echo done
