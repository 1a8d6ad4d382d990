#!/bin/bash
# PMC passes over the tail-ablation microbenchmark (tools/ntt_tail_ablation): SQ issue/wait
# counters, then TA/TD busy and stall counters, one pass each.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tail_pmc && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/tail_pmc/sq -o run -- ./tools/ntt_tail_ablation > gpurun_out/tail_pmc/sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/tail_pmc/sq.log; exit 1; }
echo sq ok
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/tail_pmc/ta -o run -- ./tools/ntt_tail_ablation > gpurun_out/tail_pmc/ta.log 2>&1 || { echo "ta pass failed"; tail -5 gpurun_out/tail_pmc/ta.log; exit 1; }
echo ta ok
