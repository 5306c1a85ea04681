set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 60 --warmup 5 --no-other-configs --no-cpu-baseline --probe"
for cfg in 64 64k; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_fetch -o p -- $B --config $cfg > gpurun_out/pmc_${cfg}_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${cfg}_write -o p -- $B --config $cfg > gpurun_out/pmc_${cfg}_write.log 2>&1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_64 -o p -- $B --config 64 > gpurun_out/kt_64.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_64_sq -o p -- $B --config 64 > gpurun_out/pmc_64_sq.log 2>&1
