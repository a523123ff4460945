#!/bin/bash
# Round 6, VERDICT r05 item 3: does a slow placement concentrate the pass's
# writes on fewer L2 channels?  place_micro quick mode (per buffer: the
# pass-shaped write V0 and a flat write) timed, then under rocprofv3 with the
# memory-side write requests split per L2 channel (TCC instance, summed over
# the XCDs) and per XCD, from one hardware counter each (derived counters,
# profiles/r06/chan_counters.yaml).
set -o pipefail
R=$GRAFT_REPO_ROOT
M=$R/mlir-hashjoin_amd/micro/bin/place_micro
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
timeout -k 10 120 $M 12 -1 1 > $O/plain.txt 2>&1 || { cat $O/plain.txt; exit 1; }
cat $O/plain.txt
cd /tmp && export TMPDIR=/tmp
Y=$R/profiles/r06/chan_counters.yaml
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum --output-format csv -d $O/pmc_dram -o run -- $M 12 -1 1 > $O/pmc_dram.log 2>&1 || { echo "pmc dram rc=$?"; tail -20 $O/pmc_dram.log; exit 1; }
I=$(python3 -c "print(' '.join('HJ_WR_I%d' % i for i in range(16)))")
timeout -s KILL 150 rocprofv3 -E $Y --pmc $I --output-format csv -d $O/pmc_inst -o run -- $M 12 -1 1 > $O/pmc_inst.log 2>&1 || { echo "pmc inst rc=$?"; tail -20 $O/pmc_inst.log; exit 1; }
X=$(python3 -c "print(' '.join('HJ_WR_X%d' % i for i in range(8)))")
timeout -s KILL 150 rocprofv3 -E $Y --pmc $X HJ_WRST_ALL --output-format csv -d $O/pmc_xcc -o run -- $M 12 -1 1 > $O/pmc_xcc.log 2>&1 || { echo "pmc xcc rc=$?"; tail -20 $O/pmc_xcc.log; exit 1; }
echo done
