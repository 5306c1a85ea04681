#!/bin/bash
# Counters for the balanced wire kernel on packed IMIX only (tools/lb_ab.py workload).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_imix
mkdir -p $O
export LB_ONLY=ipv4_lb_1M_imix_packed_verify
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/a -o p -- python3 tools/lb_ab.py > $O/a.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- python3 tools/lb_ab.py > $O/b.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 tools/lb_ab.py > $O/kt.log 2>&1
echo done
