#!/bin/bash
# One parametrised GPU driver (through gpurun, from the repo root), replacing round 3's one-off
# r3_*.sh launchers.  usage: bash tools/gpu_task.sh OUT task [task ...]; results under gpurun_out/OUT.
# Every GPU step has its own time limit; set -e ends the call at the first failure.
#   tests [-- pytest args]  the -m gpu suite (or the named test files: TESTS="tests/a.py tests/b.py")
#   smoke                   __graft_entry__.smoke()
#   bench                   the default bench line (BENCH_rNN's command)
#   c2                      the C2 leg alone, 12 steps (BENCH_ARGS overrides)
#   rocwin                  rocprofv3 --kernel-trace --stats of the C2 leg, timed window averages
#                           (tools/trace_window.py) beside the bench's own live dispatch-inclusive averages
#   pmc                     FETCH_SIZE / WRITE_SIZE passes (separate runs) over the C2 leg, reduced to
#                           per-class traffic / algorithmic bytes (tools/pmc_reduce.py)
#   pmcbench                FETCH_SIZE / WRITE_SIZE passes over the bench's C2 leg itself (not a one-round proxy)
#   rccl1                   torchrun --nproc-per-node=1 bench.py with AESFHE_FORCE_DIST=1: the RCCL process-group path
#   twogpu                  torchrun --nproc-per-node=2 bench.py --gpus 2 over gloo on ONE MI355X (both ranks
#                           share it): the N > 1 engine path at the C4 / C5 per-rank shapes
#   boot                    tools/boot_phases.py 32 (sparse bootstrap phases)
#   fhe                     tools/fhe_profile.py (true-FHE encrypt by step); FHE_ENV="A=1 B=0" runs it per setting
#   census                  tools/launch_census.py (launches / ms per AES step)
#   opcensus                tools/op_kernel_census.py (launches of one encrypt by C-ABI entry and kernel)
#   stack                   tools/step_profile.py on the 64-pair stacked leg (STACK_ARGS)
#   sweep                   tools/ntt_grid_sweep.py (NTT time vs rows per block-size configuration)
#   probes                  tools/micro/grid_sync_probe, graph_gap_probe, wt_boundary_probe (built here by hipcc)
set -e -o pipefail
O=gpurun_out/${1:?out dir}
shift
mkdir -p $O
export TMPDIR=/tmp
C2="--no-cpu-baseline --batch-states 0 --folded-steps 0 --true-fhe-steps 0 --pair-states 0 --packed-pairs 0 --eager-steps 0 --deferred-steps 0"
for t in "$@"; do
  echo "[gpu_task] $t $(date +%T)"
  case $t in
    tests)
      timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
      tail -2 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 900 python3 bench.py --detail-json $O/bench_detail.json ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err ;;
    c2)
      timeout -k 10 400 python3 bench.py --steps 12 --warmup 2 $C2 ${BENCH_ARGS:-} > $O/c2.json 2> $O/c2.err ;;
    rocwin)
      AESFHE_MARK_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
          python3 bench.py --steps 12 --warmup 2 $C2 --detail-json $O/bench_under_rocprof_detail.json > $O/bench_under_rocprof.json 2> $O/rocwin.err
      cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
      timeout -k 10 120 python3 tools/trace_window.py $O/kernel_stats_timed.json $O/prof
      rm -f $O/prof/run_kernel_trace.csv ;;
    pmc)
      # FETCH_SIZE / WRITE_SIZE passes over one middle C2 round (tools/pmc_round.py) with the
      # engine's algorithmic bytes of the same launches.  The full bench under the counters does not
      # complete on this image: with --kernel-include-regex no encrypt finished in 270 s (twice), without
      # it rocprofv3 segfaulted in its own thread 6 s in (profiles/r4_pmc_bench_attempts.txt)
      KIDS=key_inner,base_convert,ntt_cols_fwd,ntt_rows_fwd,ntt_rows_inv,ntt_cols_inv,lin_mac
      RX='k_ntt1_fwd|k_ntt2_fwd|k_ntt1_inv|k_ntt2_inv|k_lin_mac|k_base_convert|k_key_inner|k_ntt2_ki|k_bx_cols'
      AESFHE_PROFILE_FROM_START=$KIDS timeout -k 10 200 python3 tools/pmc_round.py $O/pmc_algorithmic.json > $O/pmc_alg.out
      timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_fetch -o run -- \
          python3 tools/pmc_round.py > $O/pmc_fetch.out 2> $O/pmc_fetch.err
      timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_write -o run -- \
          python3 tools/pmc_round.py > $O/pmc_write.out 2> $O/pmc_write.err
      timeout -k 10 300 python3 tools/pmc_reduce.py "--source=rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (separate runs, --kernel-include-regex on the NTT / conversion / key-switch / lin_mac kernels) over tools/pmc_round.py: one middle encrypt round of the bench workload, whole process incl. key generation; algorithmic bytes of exactly those launches from the engine (AESFHE_PROFILE_FROM_START); FETCH_SIZE x2 for 16-B-per-lane reads, x1 for NTT pass 2 dword reads (tools/ntt_pmc_calib.py); L2-miss bytes (MALL hits included), an upper bound on HBM bytes" \
          --alg=$O/pmc_algorithmic.json $O/pmc_traffic_round.json $O/pmc_fetch $O/pmc_write > /dev/null
      rm -rf $O/pmc_fetch $O/pmc_write ;;
    pmcbench)
      # FETCH_SIZE / WRITE_SIZE passes (separate runs, every kernel) over the bench's C2 leg itself
      # (bench.py --whole-stats: no sampled profiler, no precision pass), the same command once more
      # for the engine's algorithmic bytes of exactly those launches (VERDICT r4 'do this' 7)
      KIDS=key_inner,base_convert,ntt_cols_fwd,ntt_rows_fwd,ntt_rows_inv,ntt_cols_inv,lin_mac
      PB="--steps ${PMC_STEPS:-1} --warmup 1 $C2 --detail-json $O/pmcb_detail.json --whole-stats $O/ws_unused.json"
      AESFHE_PROFILE_FROM_START=$KIDS timeout -k 10 200 python3 bench.py --steps ${PMC_STEPS:-1} --warmup 1 $C2 \
          --detail-json $O/pmcb_detail0.json --whole-stats $O/pmcb_algorithmic.json > $O/pmcb_alg.out
      # HIP_ENABLE_DEFERRED_LOADING=0: every code object loaded at start-up.  With lazy loading (the default)
      # the FETCH pass died with SIGSEGV inside rocprofv3's dispatch interception at the FIRST dispatch of a
      # kernel of a not-yet-loaded translation unit (k_ntt2_inv8 r5, k_lut_bivariate / k_dec_blocksum r6:
      # a libc copy faulting at a 1 MiB-aligned address, profiles/r6_pmc_sigsegv.txt); the WRITE pass takes
      # WRITE_SIZE itself (its raw TCC_EA0_WRREQ counters hung the bench at start-up twice in round 6)
      HIP_ENABLE_DEFERRED_LOADING=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcb_fetch -o run -- \
          python3 bench.py $PB > $O/pmcb_fetch.out 2> $O/pmcb_fetch.err
      HIP_ENABLE_DEFERRED_LOADING=0 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcb_write -o run -- \
          python3 bench.py $PB > $O/pmcb_write.out 2> $O/pmcb_write.err
      timeout -k 10 300 python3 tools/pmc_reduce.py "--source=rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs, every kernel, HIP_ENABLE_DEFERRED_LOADING=0) over the bench's own C2 leg (bench.py --steps ${PMC_STEPS:-1} --warmup 1, secondary legs off), whole process; algorithmic bytes of the same launches (AESFHE_PROFILE_FROM_START); FETCH x2 for 16-B-per-lane reads, x1 for NTT pass-2 dword reads (MI355X_MICROARCH.md HBM section, tools/ntt_pmc_calib.py)" \
          --alg=$O/pmcb_algorithmic.json $O/pmc_traffic_bench.json $O/pmcb_fetch $O/pmcb_write > /dev/null
      rm -rf $O/pmcb_fetch $O/pmcb_write ;;
    twogpu)
      AESFHE_DIST_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
          --master-port=29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --batch-states 1024 --c5-states 256 \
          --pair-states 0 --packed-pairs 0 --true-fhe-steps 0 --eager-steps 0 --deferred-steps 0 > $O/bench_2rank_1gpu.json 2> $O/twogpu.err ;;
    rccl1)
      # the RCCL ("nccl") process-group path of bench.py on ONE MI355X: one rank under torch.distributed.run
      # with AESFHE_FORCE_DIST=1 (key broadcast, barriers, all_gather and max-over-ranks as GPU tensors)
      AESFHE_FORCE_DIST=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
          --master-port=29531 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --batch-states 256 --c5-states 256 \
          --pair-states 0 --packed-pairs 0 --true-fhe-steps 0 --eager-steps 0 --deferred-steps 0 > $O/bench_rccl_1rank.json 2> $O/rccl1.err ;;
    boot)
      timeout -k 10 300 python3 tools/boot_phases.py 32 ${BOOT_SET:-7 4} > $O/boot_phases.json 2> $O/boot.err ;;
    fhe)
      for e in ${FHE_ENV:-AESFHE_NONE=0}; do
        env $e timeout -k 10 300 python3 tools/fhe_profile.py ${FHE_ARGS:-2} > $O/fhe_profile_$e.json 2> $O/fhe_$e.err
        cat $O/fhe_profile_$e.json
      done ;;
    census)
      timeout -k 10 300 python3 tools/launch_census.py > $O/launch_census.json 2> $O/census.err ;;
    opcensus)
      AESFHE_CENSUS=1 timeout -k 10 300 python3 tools/op_kernel_census.py > $O/op_kernel_census.json 2> $O/opcensus.err ;;
    stack)
      timeout -k 10 600 python3 tools/step_profile.py ${STACK_ARGS:-pairs=64 reps=1} > $O/stack_profile.json 2> $O/stack.err ;;
    sweep)
      timeout -k 10 600 python3 tools/ntt_grid_sweep.py > $O/ntt_grid_sweep.json 2> $O/sweep.err ;;
    probes)
      timeout -k 10 120 tools/micro/grid_sync_probe > $O/grid_sync_probe.json
      timeout -k 10 120 tools/micro/graph_gap_probe > $O/graph_gap_probe.json
      timeout -k 10 120 tools/micro/wt_boundary_probe > $O/wt_boundary_probe.json ;;
    *) echo "unknown task $t"; exit 2 ;;
  esac
done
echo "[gpu_task] done $(date +%T)"
