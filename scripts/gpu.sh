#!/bin/bash
# One parametrised wrapper for the GPU box (run through gpurun from the repo root):
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Output under gpurun_out/TAG/.  Every GPU step runs under its own `timeout -k`; the steps are
# chained and the script stops at the first failure (no GPU step after a fault, abort or time
# limit).  Steps:
#   tests      the whole `pytest -m gpu` suite (GPU_TESTS="tests/test_x.py ..." selects files,
#              GPU_K="expr" a -k filter)
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (-> bench.json; extra args in BENCH_ARGS)
#   profile    one `rocprofv3 --kernel-trace --stats` pass per bench leg (bench.py --legs L), then
#              the PMC passes: FETCH_SIZE and WRITE_SIZE of the C3 fit and of the path-0 build,
#              the MFMA-busy counters of the C3 and C4 factorisations.  scripts/profile_collect.py
#              TAG turns the output into the profiles/TAG_<leg>_* summaries bench.py attaches.
#   shared     the N = 2 bench path rehearsed on one GPU (two processes, gloo + peer context)
#   peer       two-process sharded-fit tests (tests/test_gpu_dist.py -k peer)
#   trace      the tile-engine timelines at N = 4096 and 16384 (scripts/pt_trace.py)
#   diag       the isolated diagonal-factor microbenchmark (scripts/diag_bench.py)
#   dist       the sharded fit on 1/2/4/8 virtual ranks (scripts/dist_time.py)
#   ab         same-box A/B of the C3 bench leg: every tools/ab/*.so (GPRX_LIB_OVERRIDE) and this
#              tree's library, alternated twice (AB_ARGS: extra bench args)
#   distab     the same for the sharded fit on 1 and 8 virtual ranks
#   envab      same-box A/B of environment settings: AB_ENVS="- GPRX_X=1 GPRX_Y=2" (one assignment
#              or "-" per variant), the bench legs in AB_ARGS, alternated twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$PWD
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

fail() { echo "step $1 failed (rc $2)"; tail -n 30 "$3" 2>/dev/null; exit "$2"; }

prof_leg() {  # $1 = leg: kernel trace + stats of one bench leg in its own process
    local leg=$1
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$leg" -o "$leg" \
        -- python3 "$R/bench.py" --legs "$leg" --cpu-n 0 --cpu-lml-ns "" --cpu-predict-q 0 > "$O/prof_$leg.json" 2> "$O/prof_$leg.err") \
        || fail "profile:$leg" $? "$O/prof_$leg.err"
    echo "profile $leg ok"
}

pmc_leg() {  # $1 = leg, $2 = output name, $3.. = counters (one block-limited pass)
    local leg=$1 name=$2
    shift 2
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o "$name" \
        -- python3 "$R/bench.py" --legs "$leg" --cpu-n 0 --cpu-lml-ns "" --cpu-predict-q 0 --steps 2 --warmup 1 --build-iters 2 \
        > "$O/$name.json" 2> "$O/$name.err") || fail "pmc:$name" $? "$O/$name.err"
    echo "pmc $name ok"
}

for step in "$@"; do
    case $step in
    tests)
        timeout -k 10 1000 python -u -m pytest ${GPU_TESTS:-tests} -m gpu -x -q ${GPU_K:+-k "$GPU_K"} \
            --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1 || fail tests $? "$O/gputest.log"
        tail -n 2 "$O/gputest.log"
        ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
            > "$O/smoke.log" 2>&1 || fail smoke $? "$O/smoke.log"
        tail -n 2 "$O/smoke.log"
        ;;
    bench)
        timeout -k 10 600 python -u bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" \
            || fail bench $? "$O/bench.err"
        python scripts/bench_brief.py "$O/bench.json"
        ;;
    profile)
        for leg in c3 predict variance lml build c2 c4 c5; do prof_leg $leg; done
        pmc_leg c3 pmcf_c3 FETCH_SIZE
        pmc_leg c3 pmcw_c3 WRITE_SIZE
        pmc_leg build pmcf_build FETCH_SIZE
        pmc_leg build pmcw_build WRITE_SIZE
        pmc_leg c3 pmcm_c3 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
        pmc_leg c4 pmcm_c4 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
        # the predict kernel's issue split (bench.py attaches it as predict.pmc)
        pmc_leg predict pmcp1_predict SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
            SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
        pmc_leg predict pmcp2_predict SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
            SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
        python scripts/pmc_generic.py "$O/predict_pmc.json" "$O/pmcp1_predict" "$O/pmcp2_predict" --kernel predict
        ;;
    shared)
        GPRX_DIST_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 100)) bench.py --gpus 2 \
            > "$O/shared_bench.json" 2> "$O/shared_bench.err" || fail shared $? "$O/shared_bench.err"
        python scripts/bench_brief.py "$O/shared_bench.json"
        ;;
    spawn)  # the driver's N > 1 command as it is (bench.py --gpus N, no launcher, default legs),
            # rehearsed with SPAWN_N (default 2) ranks sharing this one GPU
        GPRX_DIST_SHARED_GPU=1 timeout -k 10 900 python bench.py --gpus ${SPAWN_N:-2} $SPAWN_ARGS \
            > "$O/spawn_bench.json" 2> "$O/spawn_bench.err" || fail spawn $? "$O/spawn_bench.err"
        python scripts/bench_brief.py "$O/spawn_bench.json"
        ;;
    peer)
        timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -k peer \
            --timeout 600 --timeout-method thread > "$O/peer.log" 2>&1 || fail peer $? "$O/peer.log"
        tail -n 2 "$O/peer.log"
        ;;
    trace)
        timeout -k 10 120 python scripts/pt_trace.py 4096 > "$O/pt4096.json" 2> "$O/pt4096.err" || fail trace $? "$O/pt4096.err"
        timeout -k 10 120 python scripts/pt_trace.py 16384 > "$O/pt16384.json" 2> "$O/pt16384.err" || fail trace $? "$O/pt16384.err"
        ;;
    diag)
        timeout -k 10 120 python scripts/diag_bench.py > "$O/diag_bench.json" 2> "$O/diag_bench.err" || fail diag $? "$O/diag_bench.err"
        ;;
    probe)  # the tile mainloop alone per operand-feed variant (tools/probe/mma_probe*, built from scripts/mma_probe.hip)
        for f in tools/probe/mma_probe*; do
            for dt in f32 f64; do
                for mode in 0 1; do
                    timeout -k 10 60 "$f" $dt 4096 10 $mode 2> "$O/probe.err" | sed "s/^{/{\"bin\": \"$(basename "$f")\", /" >> "$O/mma_probe.jsonl" || fail probe $? "$O/probe.err"
                done
            done
        done
        cat "$O/mma_probe.jsonl"
        ;;
    dist)
        timeout -k 10 300 python scripts/dist_time.py > "$O/dist_time.jsonl" 2> "$O/dist_time.err" || fail dist $? "$O/dist_time.err"
        ;;
    ab)
        shopt -s nullglob
        Q="--cpu-n 0 --cpu-predict-q 0 --legs c3 --steps 20 $AB_ARGS"
        for rep in 1 2; do
            for f in tools/ab/*.so; do
                b=$(basename "$f" .so)
                GPRX_LIB_OVERRIDE=$R/$f timeout -k 10 300 python bench.py $Q > "$O/ab_${b}_$rep.json" 2> "$O/ab.err" \
                    || fail ab $? "$O/ab.err"
            done
            timeout -k 10 300 python bench.py $Q > "$O/ab_tree_$rep.json" 2> "$O/ab.err" || fail ab $? "$O/ab.err"
        done
        for f in "$O"/ab_*.json; do echo "$(basename "$f") $(python scripts/bench_brief.py "$f" | head -1)"; done
        ;;
    distab)
        shopt -s nullglob
        for f in tools/ab/*.so; do
            b=$(basename "$f" .so)
            GPRX_LIB_OVERRIDE=$R/$f timeout -k 10 300 python -u scripts/dist_time.py 16384 5 v1 v8 > "$O/distab_$b.jsonl" \
                2> "$O/distab.err" || fail distab $? "$O/distab.err"
        done
        timeout -k 10 300 python -u scripts/dist_time.py 16384 5 v1 v8 > "$O/distab_tree.jsonl" 2> "$O/distab.err" \
            || fail distab $? "$O/distab.err"
        ;;
    envab)
        Q="--cpu-n 0 --cpu-predict-q 0 --legs c3 --steps 20 $AB_ARGS"
        for rep in 1 2; do
            for v in $AB_ENVS; do
                b=$(echo "$v" | tr '=/' '__')
                if [ "$v" = "-" ]; then
                    timeout -k 10 300 python bench.py $Q > "$O/envab_base_$rep.json" 2> "$O/envab.err" || fail envab $? "$O/envab.err"
                else
                    env $(echo "$v" | tr "," " ") timeout -k 10 300 python bench.py $Q > "$O/envab_${b}_$rep.json" 2> "$O/envab.err" \
                        || fail envab $? "$O/envab.err"
                fi
            done
        done
        for f in "$O"/envab_*.json; do echo "$(basename "$f")"; python scripts/bench_brief.py "$f" | head -4; done
        ;;
    predpmc)  # the predict kernel's issue split: two SQ passes
        (timeout -k 10 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1) || true
        pmc_leg predict pmcp1_predict SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
            SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
        pmc_leg predict pmcp2_predict SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE \
            SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
        pmc_leg predict pmcp3_predict SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
            SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU GRBM_GUI_ACTIVE
        python scripts/pmc_generic.py "$O/predict_pmc.json" "$O/pmcp1_predict" "$O/pmcp2_predict" "$O/pmcp3_predict" \
            --kernel predict
        ;;
    predmix)  # the instruction mix alone (one pass)
        pmc_leg predict pmcp3_predict SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
            SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU GRBM_GUI_ACTIVE
        python scripts/pmc_generic.py "$O/predict_mix.json" "$O/pmcp3_predict" --kernel predict
        ;;
    lmlpmc)  # the LML leg's kernels: MFMA busy and the wait split
        pmc_leg lml pmcl1_lml SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
            SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
        python scripts/pmc_generic.py "$O/lml_pmc.json" "$O/pmcl1_lml"
        ;;
    pairtrace)  # bare factorisation timelines with and without paired updates (f64 16384, f32 32768)
        for pr in 0 4; do
            GPRX_PT_PAIR=$pr timeout -k 10 120 python scripts/pt_trace.py 16384 > "$O/pt16384_pair$pr.json" \
                2> "$O/pt_pair.err" || fail pairtrace $? "$O/pt_pair.err"
            GPRX_PT_PAIR=$pr PT_TRACE_DTYPE=0 timeout -k 10 180 python scripts/pt_trace.py 32768 > "$O/pt32768f_pair$pr.json" \
                2> "$O/pt_pair.err" || fail pairtrace $? "$O/pt_pair.err"
        done
        ;;
    fittrace)  # the C3 fit's tile timeline (fused build), for the launch decomposition
        PT_TRACE_FIT=1 PT_TRACE_OUT="$O/pt_fit16384.npz" timeout -k 10 120 python scripts/pt_trace.py 16384 \
            > "$O/pt_fit16384.json" 2> "$O/pt_fit16384.err" || fail fittrace $? "$O/pt_fit16384.err"
        ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "all steps done"
