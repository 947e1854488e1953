#!/bin/bash
# rocprofv3 passes over bench.py (one gpurun call). Pass 1: kernel trace + stats. Passes 2-3:
# PMC counters, one block of counters per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass
# on gfx950), each with --kernel-trace only. Outputs under gpurun_out/prof_*; summaries are then
# copied into profiles/ by hand.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --cpu-spp 0 --no-stats --david-spp 0"}
# PROG overrides the profiled program (default bench.py), e.g. PROG="tools/render_once.py david 960 540 16"
PROG=${PROG:-"bench.py $BENCH_ARGS"}
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  case $rc in 0) return 0;; *) echo "stopping after rc=$rc"; exit $rc;; esac
}
PASSES=${PASSES:-"list trace fetch write valu"}
for p in $PASSES; do
  case $p in
    list)  step ${PFX:-}prof_list 120 rocprofv3 -L ;;
    trace) step ${PFX:-}prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${PFX:-}prof_trace" -o run -- python3 $REPO/$PROG ;;
    fetch) step ${PFX:-}prof_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/${PFX:-}prof_fetch" -o run -- python3 $REPO/$PROG ;;
    write) step ${PFX:-}prof_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/${PFX:-}prof_write" -o run -- python3 $REPO/$PROG ;;
    stall) step ${PFX:-}prof_stall 600 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/${PFX:-}prof_stall" -o run -- python3 $REPO/$PROG ;;
    mix)   step ${PFX:-}prof_mix 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT --output-format csv -d "$OUT/${PFX:-}prof_mix" -o run -- python3 $REPO/$PROG ;;
    mem)   step ${PFX:-}prof_mem 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INST_CYCLES_SMEM SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CU_CYCLES --output-format csv -d "$OUT/${PFX:-}prof_mem" -o run -- python3 $REPO/$PROG ;;
    icache) step ${PFX:-}prof_icache 600 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d "$OUT/${PFX:-}prof_icache" -o run -- python3 $REPO/$PROG ;;
    cache) step ${PFX:-}prof_cache 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/${PFX:-}prof_cache" -o run -- python3 $REPO/$PROG ;;
    ta)    step ${PFX:-}prof_ta 600 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum --output-format csv -d "$OUT/${PFX:-}prof_ta" -o run -- python3 $REPO/$PROG ;;
    tcp)   step ${PFX:-}prof_tcp 600 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/${PFX:-}prof_tcp" -o run -- python3 $REPO/$PROG ;;
    lds)   step ${PFX:-}prof_lds 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d "$OUT/${PFX:-}prof_lds" -o run -- python3 $REPO/$PROG ;;
    valu)  step ${PFX:-}prof_valu 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/${PFX:-}prof_valu" -o run -- python3 $REPO/$PROG ;;
  esac
done
