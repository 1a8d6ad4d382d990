#!/bin/bash
# Where the NTT passes lose issue slots: wave-state PMC pass (active / waiting / issue-stalled
# quad-cycles) and LDS counters over one C3 commit.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_stall
mkdir -p $OUT
B="python3 bench.py --config C3 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- $B --steps 1 --warmup 0 > $OUT/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $OUT/sq.log; exit 1; }
echo sq ok
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $OUT/lds -o run -- $B --steps 1 --warmup 0 > $OUT/lds.log 2>&1 || { echo "lds rc=$?"; tail -5 $OUT/lds.log; exit 1; }
echo lds ok
