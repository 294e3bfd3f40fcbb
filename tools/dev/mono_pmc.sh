# Dev (GPU box, repo root): TCC counters over tools/dev/alloc_modes.py, one
# rocprofv3 --pmc pass per counter set; the allocations land in either speed
# mode, so every pass sees both.  tools/dev/mono_pmc.sh [line]
set -o pipefail
LINE=${1:-m24to48}
cd /tmp && export TMPDIR=/tmp REALLOCS=8
O=$GRAFT_REPO_ROOT/gpurun_out/mmp/$LINE; mkdir -p $O
P="python3 -u $GRAFT_REPO_ROOT/tools/dev/alloc_modes.py $LINE quick"
i=0
for SET in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCC_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_RDREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $SET GRBM_GUI_ACTIVE -d $O/p$i -o run --output-format csv -- $P > $O/p$i.log 2>&1 || exit 1
done
