#!/bin/bash
# One GPU session on the box (run via gpurun from the repo root):
#   gpurun -- bash scripts/gpu_run.sh <tag> <step>...
# steps (each under its own time limit, stopping at the first failure):
#   native    tests/test_gpu_native.py (native code on the reference vectors, query shapes, 2^26)
#   gpu       the whole -m gpu suite
#   noasm     the C++ step() build of the interpreter against the oracle (one test)
#   smoke     __graft_entry__.smoke()
#   bench     default bench.py (N=1)
#   miss      scripts/miss_cost.py (per-stage cost of sieve misses, JIT build vs interpreter)
#   queries   scripts/sieve_queries.py (per-query latency, LASER order and cold)
#   latency   two more passes of sieve_queries.py at 9 repetitions (sieve_queries_{a,b}.jsonl)
#   interp    scripts/interp_op_cost.py (interpreter cost of a loaded column / a complex op;
#             MH_INTERP_SC=0: its conjunctions are false on random rows, the ops are the point)
#   counters  rocprofv3 -L (the PMC counters this box offers)
#   profile   scripts/profile.sh <tag> (kernel trace + PMC passes of the default bench)
#   kbench    bench.py --variant keccak (config 4's kernel, 2^20 rows)
#   kprofile  scripts/profile.sh <tag>_keccak --variant keccak
#   paths     scripts/path_scaling.py (latency against path length, 25..400 constraints)
#   bfs       scripts/bfs_order.py --solve and host-only (BFS / JUMPI order at 400 constraints)
#   jumpi     scripts/jumpi_order.py (both branches of every JUMPI, 100 and 400 constraints)
#   ibench    bench.py --engine interp (config 5 on the interpreter, one step)
#   strong    bench.py --strong at N=1 (config 5 literally: 2^26 rows in total)
#   import    scripts/import_cost.py (the z3 import stage per new constraint, C++ vs Python)
#   pylatency latency's two passes with the Python host stages (SIEVE_HOST=python)
#   pypaths   paths with the Python host stages
#   qcost     scripts/query_cost.py (host stages per query, native compiler vs Python)
#   qprofile  rocprofv3 kernel trace + stats of one pass of sieve_queries.py (query-path kernels)
#   pprof4    pprofile for the default and variant libraries ($PV, default nowin) at first-round
#             sizes $PFR (default 256 4096)
#   bitop3    scripts/valu_peak.py for v_bitop3_b32 beside xor / alignbit / cndmask
#   valu6     scripts/valu_peak.py for the round-6 candidates (64-bit compares, v_lshl_add_u64, the
#             32-bit multiplies) beside the carry chains and v_mad_u64_u32
#   hostprof  scripts/solve_profile.py (cProfile of LASER-order queries at 400 constraints)
#   hiptrace  rocprofv3 HIP runtime + kernel trace of solve_profile.py (EtherThief-400)
#   pprofile  rocprofv3 kernel trace + stats of path_scaling.py at 400 constraints
#   gather    scripts/gather_bench.py (survivor reload cost of lane compaction, SoA vs row-major)
#   recall    scripts/planted_recall.py (recall on planted-SAT paths, per round and shape class)
#   cdreads   scripts/calldata_reads.py (the reference's calldata byte loop over a sieve model)
#   misses    scripts/recall_misses.py (first misses of the random family: search or lowering)
#   feedback  planted_recall with every miss answered by the planted model, learnt (--feedback)
#   recalli   planted_recall without the incremental second round (SIEVE_INCREMENTAL=0)
#   grecall   tests/test_gpu_recall.py with its printed numbers (-s)
#   incrows   planted_recall with 16384 / 65536-row incremental rounds (SIEVE_INC_ROWS)
#   inchops   planted_recall with the parent's column-sharing conjuncts in the incremental guide
#   inc16k    planted_recall, path_scaling and sieve_queries with 16384-row incremental rounds,
#             then path_scaling and sieve_queries at the default on the same box
#   round3    planted_recall and path_scaling with a third round (the full guide's 2^16 rows after
#             the incremental round, SIEVE_ROUND3=1), then path_scaling at the default
#   peval     planted_recall without the parent-evaluating incremental guide (SIEVE_INC_PEVAL=0)
#   recall0   planted_recall without the keccak second chance (SIEVE_KECCAK2=0), no extended pass
#   round2    planted_recall and path_scaling with the second round gated on first-round progress
#             (SIEVE_ROUND2=progress) and never run (recall only)
#   policy    sieve_queries.py (9 reps) and path_scaling.py with the second round always run and
#             gated on first-round progress (SIEVE_ROUND2=always / progress), back to back
#   nopf      interp, paths and queries (9 reps) on the variant library built without the
#             interpreter's LOADVAR prefetch (scripts/build_variant.sh nopf MH_GEN_LV_PREFETCH=0)
#   ab_<v>    the same on any variant library mythril_amd/libmythril_hip_<v>.so
#             (scripts/build_variant.sh <v> GENERATOR_SWITCH=...)
#   scab      paths and queries (9 reps) with the interpreter's short-circuit conjunctions off
#             (MH_INTERP_SC=0) and in the conjuncts' given order (MH_INTERP_SC=given)
#   rows1     paths, queries (9 reps) and planted recall with first rounds of 256 / 4096 / 16384
#             rows (SIEVE_FIRST_ROWS)
#   split     paths and queries with conjunct-parallel rounds (MH_SPLIT_INSNS in $SPLITS)
#   qpmc      scripts/qprofile_pmc.sh <tag> (PMC passes of the query-path kernels)
#   qpmcnopf  the same on the no-prefetch variant library
#   occupancy bench.py at 168 and 256 VGPRs (3 and 2 waves per SIMD; the LDS-resident compaction
#             design of DESIGN §10 needs one of them)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    native)   timeout -k 10 1000 $PYT tests/test_gpu_native.py > "$OUT/pytest_native.txt" 2>&1 ;;
    noasm)    timeout -k 10 400 $PYT -m gpu tests/test_gpu_parity.py -k cpp_step_build > "$OUT/pytest_noasm.txt" 2>&1 ;;
    gpu)      timeout -k 10 1100 $PYT -m gpu tests > "$OUT/pytest_gpu.txt" 2>&1 ;;
    smoke)    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 ;;
    bench)    timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.log" ;;
    miss)     timeout -k 10 400 python -u scripts/miss_cost.py 5 > "$OUT/miss_cost.jsonl" 2> "$OUT/miss_cost.log" ;;
    queries)  timeout -k 10 400 python -u scripts/sieve_queries.py > "$OUT/sieve_queries.jsonl" 2> "$OUT/sieve_queries.log" ;;
    latency)  SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py \
                > "$OUT/sieve_queries_a.jsonl" 2> "$OUT/a.log" && \
              SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py \
                > "$OUT/sieve_queries_b.jsonl" 2> "$OUT/b.log" ;;
    interp)   MH_INTERP_SC=0 timeout -k 10 300 python -u scripts/interp_op_cost.py > "$OUT/interp_op_cost.jsonl" 2> "$OUT/interp_op_cost.log" ;;
    counters) timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 ;;
    profile)  bash scripts/profile.sh "$TAG" ;;
    kbench)   timeout -k 10 400 python -u bench.py --variant keccak --cpu-seconds 5 > "$OUT/bench_keccak.json" 2> "$OUT/bench_keccak.log" ;;
    kprofile) bash scripts/profile.sh "${TAG}_keccak" --variant keccak ;;
    paths)    timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling.jsonl" 2> "$OUT/path_scaling.log" ;;
    bfs)      timeout -k 10 600 python -u scripts/bfs_order.py --solve > "$OUT/bfs_order_solve.jsonl" 2> "$OUT/bfs_order_solve.log" && \
              timeout -k 10 300 python -u scripts/bfs_order.py > "$OUT/bfs_order_host.jsonl" 2> "$OUT/bfs_order_host.log" ;;
    jumpi)    timeout -k 10 600 python -u scripts/jumpi_order.py > "$OUT/jumpi_order.jsonl" 2> "$OUT/jumpi_order.log" ;;
    import)   timeout -k 10 300 python -u scripts/import_cost.py > "$OUT/import_cost.jsonl" 2> "$OUT/import_cost.log" ;;
    ibench)   timeout -k 10 600 python -u bench.py --engine interp --steps 1 --warmup 1 --no-companion --no-cpu-baseline > "$OUT/bench_interp.json" 2> "$OUT/bench_interp.log" ;;
    strong)   timeout -k 10 400 python -u bench.py --strong --no-companion --cpu-seconds 3 > "$OUT/bench_strong.json" 2> "$OUT/bench_strong.log" ;;
    pylatency) SIEVE_HOST=python SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py \
                > "$OUT/sieve_queries_py_a.jsonl" 2> "$OUT/py_a.log" && \
              SIEVE_HOST=python SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py \
                > "$OUT/sieve_queries_py_b.jsonl" 2> "$OUT/py_b.log" ;;
    pypaths)  SIEVE_HOST=python timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_py.jsonl" 2> "$OUT/path_scaling_py.log" ;;
    recall)   timeout -k 10 900 python -u scripts/planted_recall.py 100 24 --extended > "$OUT/planted_recall.jsonl" 2> "$OUT/planted_recall.log" ;;
    occupancy) MH_JIT_PAD_VGPR=168 timeout -k 10 400 python -u bench.py --no-companion --no-cpu-baseline --steps 2 > "$OUT/bench_vgpr168.json" 2> "$OUT/bench_vgpr168.log" && \
              MH_JIT_PAD_VGPR=256 timeout -k 10 400 python -u bench.py --no-companion --no-cpu-baseline --steps 2 > "$OUT/bench_vgpr256.json" 2> "$OUT/bench_vgpr256.log" ;;
    cdreads)  timeout -k 10 300 python -u scripts/calldata_reads.py > "$OUT/calldata_reads.json" 2> "$OUT/calldata_reads.log" ;;
    misses)   timeout -k 10 600 python -u scripts/recall_misses.py 100 24 > "$OUT/recall_misses.json" 2> "$OUT/recall_misses.log" ;;
    feedback) timeout -k 10 600 python -u scripts/planted_recall.py 100 24 --feedback > "$OUT/planted_recall_feedback.jsonl" 2> "$OUT/planted_recall_feedback.log" ;;
    recalli)  SIEVE_INCREMENTAL=0 timeout -k 10 900 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_noinc.jsonl" 2> "$OUT/planted_recall_noinc.log" ;;
    grecall)  timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_recall.py > "$OUT/pytest_recall.txt" 2>&1 ;;
    incrows)  for r in 16384 65536; do SIEVE_INC_ROWS=$r timeout -k 10 600 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_inc$r.jsonl" 2> "$OUT/planted_recall_inc$r.log" || exit 1; done ;;
    inchops)  SIEVE_INC_HOPS=1 timeout -k 10 600 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_hops1.jsonl" 2> "$OUT/planted_recall_hops1.log" ;;
    inc16k)   SIEVE_INC_ROWS=16384 timeout -k 10 600 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_inc16k.jsonl" 2> "$OUT/planted_recall_inc16k.log" && \
              SIEVE_INC_ROWS=16384 timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_inc16k.jsonl" 2> "$OUT/path_scaling_inc16k.log" && \
              SIEVE_INC_ROWS=16384 SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_inc16k.jsonl" 2> "$OUT/sieve_queries_inc16k.log" && \
              timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling.jsonl" 2> "$OUT/path_scaling.log" && \
              SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries.jsonl" 2> "$OUT/sieve_queries.log" ;;
    round3)   SIEVE_ROUND3=1 timeout -k 10 600 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_r3.jsonl" 2> "$OUT/planted_recall_r3.log" && \
              SIEVE_ROUND3=1 timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_r3.jsonl" 2> "$OUT/path_scaling_r3.log" && \
              timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling.jsonl" 2> "$OUT/path_scaling.log" ;;
    peval)    SIEVE_INC_PEVAL=0 timeout -k 10 600 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_nopeval.jsonl" 2> "$OUT/planted_recall_nopeval.log" ;;
    recall0)  SIEVE_KECCAK2=0 timeout -k 10 900 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_nok2.jsonl" 2> "$OUT/planted_recall_nok2.log" ;;
    round2)   timeout -k 10 600 python -u scripts/planted_recall.py 100 24 --round2=progress > "$OUT/planted_recall_progress.jsonl" 2> "$OUT/planted_recall_progress.log" && \
              timeout -k 10 600 python -u scripts/planted_recall.py 100 24 --round2=never > "$OUT/planted_recall_never.jsonl" 2> "$OUT/planted_recall_never.log" && \
              SIEVE_ROUND2=progress timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_progress.jsonl" 2> "$OUT/path_scaling_progress.log" ;;
    policy)   for pol in always progress; do \
                SIEVE_ROUND2=$pol SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_$pol.jsonl" 2> "$OUT/sieve_queries_$pol.log" && \
                SIEVE_ROUND2=$pol timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_$pol.jsonl" 2> "$OUT/path_scaling_$pol.log" || exit 1; done ;;
    nopf|ab_*) V=${step#ab_}; export MYTHRIL_HIP_LIB=$PWD/mythril_amd/libmythril_hip_$V.so && \
              MH_INTERP_SC=0 timeout -k 10 300 python -u scripts/interp_op_cost.py > "$OUT/interp_op_cost_$V.jsonl" 2> "$OUT/interp_op_cost_$V.log" && \
              timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_$V.jsonl" 2> "$OUT/path_scaling_$V.log" && \
              SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_$V.jsonl" 2> "$OUT/sieve_queries_$V.log"; \
              rc=$?; unset MYTHRIL_HIP_LIB; (exit $rc) ;;
    scab)     for sc in 0 given; do \
                MH_INTERP_SC=$sc timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_sc$sc.jsonl" 2> "$OUT/path_scaling_sc$sc.log" && \
                MH_INTERP_SC=$sc SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_sc$sc.jsonl" 2> "$OUT/sieve_queries_sc$sc.log" || exit 1; done ;;
    rows1)    for fr in 256 4096 16384; do \
                SIEVE_FIRST_ROWS=$fr timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_fr$fr.jsonl" 2> "$OUT/path_scaling_fr$fr.log" && \
                SIEVE_FIRST_ROWS=$fr SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_fr$fr.jsonl" 2> "$OUT/sieve_queries_fr$fr.log" && \
                SIEVE_FIRST_ROWS=$fr timeout -k 10 900 python -u scripts/planted_recall.py 100 24 > "$OUT/planted_recall_fr$fr.jsonl" 2> "$OUT/planted_recall_fr$fr.log" || exit 1; done ;;
    split)    for si in ${SPLITS:-384 1024}; do \
                MH_SPLIT_INSNS=$si timeout -k 10 600 python -u scripts/path_scaling.py > "$OUT/path_scaling_split$si.jsonl" 2> "$OUT/path_scaling_split$si.log" && \
                MH_SPLIT_INSNS=$si SIEVE_QUERY_REPS=9 timeout -k 10 300 python -u scripts/sieve_queries.py > "$OUT/sieve_queries_split$si.jsonl" 2> "$OUT/sieve_queries_split$si.log" || exit 1; done ;;
    qpmc)     bash scripts/qprofile_pmc.sh "$TAG" ;;
    qpmc256)  SIEVE_FIRST_ROWS=256 bash scripts/qprofile_pmc.sh "${TAG}_256" ;;
    qpmcnopf) MYTHRIL_HIP_LIB=$PWD/mythril_amd/libmythril_hip_nopf.so bash scripts/qprofile_pmc.sh "${TAG}_nopf" ;;
    qcost)    timeout -k 10 300 python -u scripts/query_cost.py > "$OUT/query_cost.jsonl" 2> "$OUT/query_cost.log" ;;
    qprofile) MH_TRACE_COMPILE=1 SIEVE_QUERY_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/qprof" -o qprof -- \
                python -u scripts/sieve_queries.py > "$OUT/qprof.jsonl" 2> "$OUT/qprof.log" ;;
    pprof4)   for v in "" ${PV:-nowin}; do for fr in ${PFR:-256 4096}; do \
                lib=$PWD/mythril_amd/libmythril_hip${v:+_$v}.so; tag=pprof${v:+_$v}_fr$fr; \
                MYTHRIL_HIP_LIB=$lib SIEVE_FIRST_ROWS=$fr timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o $tag -- \
                  python -u scripts/path_scaling.py 400 > "$OUT/$tag.jsonl" 2> "$OUT/$tag.log" || exit 1; done; done ;;
    bitop3)   timeout -k 10 300 python -u scripts/valu_peak.py bitop3_b32 mix_bitop3_alignbit xor_b32 alignbit_b32 cndmask_b32 > "$OUT/valu_bitop3.json" 2> "$OUT/valu_bitop3.log" ;;
    valu6)    timeout -k 10 300 python -u scripts/valu_peak.py cmp_lt_u64 cmp_eq_u64 lshl_add_u64 mul_lo_u32 mul_hi_u32 \
                mul_u32_u24 sub_co_e64_sgpr cmp_lt_u32_e64 lt256_via_u64 add_co_chain sub_co_vcc_chain mad_u64_u32 \
                cmp_eq_e32 xor_b32 bitop3_b32 or3_b32 > "$OUT/valu6.json" 2> "$OUT/valu6.log" ;;
    hostprof) timeout -k 10 300 python -u scripts/solve_profile.py ether_thief 400 40 > "$OUT/solve_profile_et400.txt" 2>&1 && \
              timeout -k 10 300 python -u scripts/solve_profile.py killbilly 400 40 > "$OUT/solve_profile_kb400.txt" 2>&1 ;;
    hiptrace) timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d "$OUT/htrace" -o htrace -- \
                python -u scripts/solve_profile.py ether_thief 400 40 > "$OUT/htrace.txt" 2> "$OUT/htrace.log" ;;
    pprofile) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pprof" -o pprof -- \
                python -u scripts/path_scaling.py 400 > "$OUT/pprof.jsonl" 2> "$OUT/pprof.log" ;;
    gather)   timeout -k 10 300 python -u scripts/gather_bench.py > "$OUT/gather.jsonl" 2> "$OUT/gather.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
