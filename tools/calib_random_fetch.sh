#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for random line traffic (MI355X_MICROARCH.md §HBM: only wide
# coalesced streaming reads are calibrated — FETCH_SIZE is half their bytes). tools/rand_gather.hip
# issues a known count of accesses (2^25 threads x 16 per launch, one warm-up + 5 timed launches per
# argument): "<gb>" independent 4-B loads at pseudo-random 64-B-aligned offsets (K1F's probes, K4's
# run-index / record reads), "n<gb>" the same loads non-temporal, "s<gb>" a coalesced 16-B-per-lane
# stream (the guide's calibrated case), "w<gb>" random 16-B stores (K4's match writes). Per dispatch:
# FETCH_SIZE / WRITE_SIZE and the L2's memory-side requests by size, against the access count.
# Output: gpurun_out/r05/calib/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/calib
mkdir -p $O
ARGS="${CALIB_ARGS:-5.4 144 n5.4 n144 s40 w144}"
timeout -k 10 120 tools/_rand_gather $ARGS > $O/timing.jsonl
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- tools/_rand_gather $ARGS > /dev/null 2> $O/fetch.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -f csv -d $O/req -o run -- tools/_rand_gather $ARGS > /dev/null 2> $O/req.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum -f csv -d $O/req2 -o run -- tools/_rand_gather $ARGS > /dev/null 2> $O/req2.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/write -o run -- tools/_rand_gather $ARGS > /dev/null 2> $O/write.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -f csv -d $O/wreq -o run -- tools/_rand_gather $ARGS > /dev/null 2> $O/wreq.log
python3 tools/calib_summary.py $O > $O/summary.json
