#!/bin/bash
# dev/lab.sh -- the one lab runner for GPU sessions (gpurun): `bash dev/lab.sh <experiment> [args]`.
# Every GPU step runs under its own timeout; the script stops at the first crash / timeout (a plain
# test failure, pytest rc 1, does not stop it). Output goes to gpurun_out/. The dev/*_lab binaries
# are built on the CPU side first (the command in each file's header); dev/README.md says which
# DESIGN.md claim each lab backs.
#
#   floors           round 6: production scatter passes with / without their stores (dev/floor_lab[_ns]), the C2
#                    and pairs write-stream floors (dev/ceiling_lab c2 / pairs), the C2 / C4 bench lines
#   round            pytest -m gpu (all) + the default bench line (what the driver runs at round end)
#   tests [-k EXPR]  pytest -m gpu, optionally filtered
#   nodes NODE...    pytest -m gpu on these files / node ids only (-s; LAB_TAG names gpurun_out/nodes_TAG.log)
#   pairs            the pairs tests + C4 and Zipf keys through bench.py, then C4 with the 64-B-line
#                    pairs kernel (RSORT_PAIRS64=1) for A/B on the same box
#   pairslab         dev/pairs_lab: one pairs pass, 64-B vs 128-B kernels, per-phase cycles
#   cl               the clustered-pass ranking A/B: Zipf keys and C4 through bench.py with RSORT_CL=1
#                    (rank_add_hot) and the default (rank_add_runs)
#   lines            dev/lines_exp: the keys line-kernel variants, uniform passes 0/1, Zipf passes 0..3
#   zcl              dev/lines_exp "pad": clustered-kernel rank variants, uniform pass 0, Zipf passes 1, 2
#   bench [args]     bench.py with extra args (LAB_TAG names the output)
#   kt TAG [args]    rocprofv3 per-launch kernel trace of a short bench run (gpurun_out/kt_TAG;
#                    dev/ktall.py / dev/ktsum.py read it)
#   variants V...    dev/var_V.so (dev/build_variant.sh) over the box's librsort.so in turn: kernel
#                    traces of the C3, Zipf-keys and all-equal benches
#   ab V [CONFIGS]   the C3 line and the configs block (default zipf,c4): the built librsort.so and
#                    dev/var_V.so (dev/build_variant.sh; e.g. HEAD's kernels), alternating twice
#   envab KV [CONFIGS] the C3 line and the configs block (default c2) with and without the library
#                    environment setting KV (e.g. RSORT_NX_TAIL=1), alternating twice
#   wgt [args]       per-workgroup durations of each scatter pass, slowest chunks of pass 1 (dev/wgtimes_lab.py)
#   sqzipf           SQ counters per pass of a Zipf-keys sort (LDS address / bank conflicts), in issue order
#   pfloor           the pairs pass's write-stream floor (dev/ceiling_lab pairs) beside the pairs kernel, one box
#   sqpmc            SQ counters (three passes) of a pairs pass (dev/pairs_lab) and a C3 sort (dev/sqpmc.py)
#   prof TAG [args]  profiles/run_profiles.sh (kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes)
#   pmc              memory-pipe PMC of rs_scatter_lines (dev/scatter_lab) vs the line-store lab (wc_lab)
#   dist             kernel trace of the multi-GPU step on one rank (bench.py --dist-path)
#   ceiling          dev/ceiling_lab: copy / read / write ceilings (policies, grids, shapes) and per-workgroup
#                    copy rates by XCC (gpurun_out/ceiling.jsonl; profiles/r05_ceilings.json)
#   wgtx             (WGTX_ARGS="..." for one run) dev/var_wgt.so: per-workgroup scatter rates of repeated sorts against XCC, physical CU
#                    and chunk (dev/wgtimes_lab.py --reps)
#   cutw             ADVICE r4: cost-weighted cut plans vs equal-count ones (RSORT_LAB=1 RSORT_CUT_WEIGHTS=0) on
#                    Zipf s=1 at 2^28 / 2^30, Zipf s=1.2 and "hot" keys at 2^30, keys and pairs, alternating twice
#   profiles TAG     the committed profile set: run_profiles.sh for C3, Zipf keys, C4 and C2 (TAG,
#                    TAG_zipf, TAG_c4, TAG_c2), then kernel traces of the one-rank multi-GPU step, the
#                    default (direct sort) and the whole protocol (--dist-full)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
exp=$1
shift
ok_or_stop() {  # pytest rc 0/1 continue, anything else (crash, timeout) stops the session
    local rc=$1
    echo "[lab] $2 rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
}
stop_unless_ok() {
    local rc=$1
    echo "[lab] $2 rc=$rc"
    [ "$rc" -eq 0 ] || exit "$rc"
}
run_bench() {  # name, args...
    local name=$1
    shift
    timeout -k 10 300 python bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
    stop_unless_ok $? "bench $name"
    tail -c 2500 "gpurun_out/$name.json"
}
kt() {  # tag, bench args...
    local tag=$1
    shift
    rm -rf "$R/gpurun_out/kt_$tag"
    (cd /tmp && TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/kt_$tag" -- \
        python3 "$R/bench.py" --no-cpu --no-e2e --no-vendor --configs "" --steps 2 --warmup 1 "$@" \
        > "$R/gpurun_out/kt_$tag.log" 2>&1)
    stop_unless_ok $? "kt $tag"
}
case "$exp" in
floors)
    # one pass of each production scatter kernel with and without its output stores
    # (dev/floor_lab, dev/floor_lab_ns), the C2 and pairs write-stream floors (dev/ceiling_lab c2 / pairs)
    # and the bench's C2 / C4 lines, all on this one box (gpurun_out/floors.jsonl)
    : > gpurun_out/floors.jsonl
    for b in floor_lab floor_lab_ns floor_lab floor_lab_ns; do
        timeout -k 10 120 dev/$b 10 >> gpurun_out/floors.jsonl 2> gpurun_out/floors.err
        stop_unless_ok $? "$b"
    done
    timeout -k 10 120 dev/ceiling_lab 26 20 c2 >> gpurun_out/floors.jsonl 2>> gpurun_out/floors.err
    stop_unless_ok $? "ceiling c2"
    timeout -k 10 200 dev/ceiling_lab 30 10 pairs >> gpurun_out/floors.jsonl 2>> gpurun_out/floors.err
    stop_unless_ok $? "ceiling pairs"
    run_bench floors_bench --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e --configs c2,c4 > /dev/null
    grep -h '"pass"\|c2_\|runs32_pairs\|runs64"' gpurun_out/floors.jsonl
    ;;
partab)
    # the multi-GPU partition (dev/part_lab.py: 2^30 keys into the buckets of N ranks) with the box's
    # librsort.so and dev/var_$1.so, alternating twice
    v=$1
    cp cuda.radixsort_amd/librsort.so gpurun_out/ab_new.so
    for side in new "$v" new "$v"; do
        if [ "$side" = new ]; then cp gpurun_out/ab_new.so cuda.radixsort_amd/librsort.so; oldlib=0
        else cp "dev/var_$v.so" cuda.radixsort_amd/librsort.so; oldlib=1; fi
        RSORT_LAB=1 RSORT_LAB_OLD_LIB=$oldlib timeout -k 10 200 python dev/part_lab.py > gpurun_out/partab_$side.log 2>&1
        stop_unless_ok $? "part_lab $side"
        echo "$side $(tail -n 1 gpurun_out/partab_$side.log)"
    done
    cp gpurun_out/ab_new.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/ab_new.so
    ;;
round)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 300 --timeout-method thread \
        > gpurun_out/round_tests.log 2>&1
    ok_or_stop $? pytest
    tail -n 3 gpurun_out/round_tests.log
    run_bench round_bench --steps 20 --warmup 5
    ;;
tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 300 --timeout-method thread "$@" \
        > gpurun_out/lab_tests.log 2>&1
    ok_or_stop $? pytest
    grep -E "passed|failed|FAILED|Error" gpurun_out/lab_tests.log | tail -n 20
    ;;
nodes)
    # pytest on the given test files / node ids only (LAB_TAG names the log), -s so prints are kept
    timeout -k 10 1000 python -u -m pytest -v -s --maxfail 8 --timeout 600 --timeout-method thread -m gpu "$@" \
        > gpurun_out/nodes_${LAB_TAG:-x}.log 2>&1
    ok_or_stop $? "pytest nodes"
    grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" gpurun_out/nodes_${LAB_TAG:-x}.log | tail -n 30
    ;;
pairs)
    timeout -k 10 600 python -u -m pytest tests -m gpu -v -k "pairs or clustered or cut_plan or group" \
        --timeout 300 --timeout-method thread > gpurun_out/pairs_tests.log 2>&1
    ok_or_stop $? pytest
    grep -E "passed|failed|FAILED|Error" gpurun_out/pairs_tests.log | tail -n 12
    run_bench pairs_new --steps 5 --warmup 2 --keys 16777216 --no-cpu --no-vendor --no-e2e --configs c4,zipf "$@"
    RSORT_LAB=1 RSORT_PAIRS64=1 run_bench pairs_64 --steps 5 --warmup 2 --keys 16777216 --no-cpu --no-vendor --no-e2e \
        --configs c4 "$@"
    ;;
pairslab)
    : > gpurun_out/pairslab.log
    for cfg in "0 0" "1 0" "1 1"; do
        set -- $cfg
        PL_ZIPF=$1 PL_PASS=$2 timeout -k 10 120 dev/pairs_lab 30 >> gpurun_out/pairslab.log 2>&1
        rc=$?
        echo "[lab] pairs_lab zipf=$1 pass=$2 rc=$rc"
        [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
    done
    cat gpurun_out/pairslab.log
    ;;
cl)
    for v in 2 1; do
        RSORT_CL=$v run_bench "cl$v" --steps 2 --warmup 1 --keys 16777216 --no-cpu --no-vendor --no-e2e \
            --configs zipf,c4 "$@" > /dev/null
        python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/cl{sys.argv[1]}.json").read().strip().splitlines()[-1])
for k, c in d["configs"].items():
    print("RSORT_CL=%s %-5s %8.3f ms/sort  scatter %.4f ms/pass (%.3f)  %s" % (sys.argv[1], k, c["ms_per_sort"],
          c["scatter"]["avg_launch_ms"], c["scatter"]["frac"], c["verified"]))
PY
    done
    ;;
lines)
    : > gpurun_out/lab_lines.log
    timeout -k 10 100 dev/lines_exp 30 "$@" >> gpurun_out/lab_lines.log 2>&1 || exit $?
    LX_PASS=1 timeout -k 10 100 dev/lines_exp 30 "$@" >> gpurun_out/lab_lines.log 2>&1 || exit $?
    for p in 0 1 2 3; do
        LX_ZIPF=1 LX_PASS=$p timeout -k 10 100 dev/lines_exp 30 "$@" >> gpurun_out/lab_lines.log 2>&1 || exit $?
    done
    cat gpurun_out/lab_lines.log
    ;;
zcl)
    : > gpurun_out/lab_zcl.log
    timeout -k 10 100 dev/lines_exp 30 "pad" >> gpurun_out/lab_zcl.log 2>&1 || exit $?
    for p in 1 2; do
        LX_ZIPF=1 LX_PASS=$p timeout -k 10 100 dev/lines_exp 30 "pad" >> gpurun_out/lab_zcl.log 2>&1 || exit $?
    done
    cat gpurun_out/lab_zcl.log
    ;;
bench)
    run_bench "bench_${LAB_TAG:-x}" "$@"
    ;;
kt)
    kt "$@"
    ;;
variants)
    for v in "$@"; do
        cp "dev/var_$v.so" cuda.radixsort_amd/librsort.so
        kt "c3_$v"
        kt "z_$v" --dist zipf
        kt "e_$v" --dist equal
    done
    ;;
ab)
    # the C3 line and bench.py's configs block (zipf, c4, or $2): the box's librsort.so ("new") and
    # dev/var_$1.so, alternating twice
    v=$1
    cp cuda.radixsort_amd/librsort.so gpurun_out/ab_new.so
    for side in new "$v" new "$v"; do
        if [ "$side" = new ]; then cp gpurun_out/ab_new.so cuda.radixsort_amd/librsort.so; else cp "dev/var_$v.so" cuda.radixsort_amd/librsort.so; fi
        # (the variant may predate symbols radixsort.py binds: RSORT_LAB_OLD_LIB leaves those unbound)
        if [ "$side" = new ]; then oldlib=0; else oldlib=1; fi
        RSORT_LAB=1 RSORT_LAB_OLD_LIB=$oldlib run_bench "ab_$side" --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e \
            --configs "${2:-zipf,c4}" > /dev/null
        python3 - "$side" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("%-6s C3    %8.3f ms/sort  scatter %.4f ms/pass (%.3f)  %s" % (sys.argv[1], d["ms_per_step"],
      r["avg_launch_ms"], r["frac"], d["verified"]))
for k, c in d["configs"].items():
    print("%-6s %-5s %8.3f ms/sort  hist %.3f  scatter %.4f ms/pass (%.3f)  %s" % (sys.argv[1], k, c["ms_per_sort"],
          c["phases_ms_per_sort"]["histogram"], c["scatter"]["avg_launch_ms"], c["scatter"]["frac"], c["verified"]))
PY
    done
    cp gpurun_out/ab_new.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/ab_new.so
    ;;
envab)
    # the C3 line and a configs block (default c2) with and without an environment setting of the
    # library, alternating twice: bash dev/lab.sh envab "RSORT_LAB=1 RSORT_NX_TAIL=1" [configs]
    kv=$1
    for side in new env new env; do
        if [ "$side" = env ]; then
            env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e \
                --configs "${2:-c2}" > gpurun_out/envab_$side.json 2> gpurun_out/envab_$side.err
        else
            timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e \
                --configs "${2:-c2}" > gpurun_out/envab_$side.json 2> gpurun_out/envab_$side.err
        fi
        stop_unless_ok $? "envab $side"
        python3 - "$side" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/envab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("%-6s C3    %8.3f ms/sort  scatter %.4f ms/pass (%.3f)  %s" % (sys.argv[1], d["ms_per_step"],
      r["avg_launch_ms"], r["frac"], d["verified"]))
for k, c in d["configs"].items():
    print("%-6s %-5s %8.3f ms/sort  hist %.3f  scatter %.4f ms/pass (%.3f)  %s %s" % (sys.argv[1], k, c["ms_per_sort"],
          c["phases_ms_per_sort"]["histogram"], c["scatter"]["avg_launch_ms"], c["scatter"]["frac"], c["verified"],
          c["plan_check"]))
PY
    done
    ;;
sqpmc)
    # SQ counters of one C4-shaped pairs pass (dev/pairs_lab, 2^29 pairs) and of a C3 sort (bench.py,
    # 2^29 keys): three passes of <= 8 SQ counters each; dev/sqpmc.py summarises gpurun_out/sqpmc_*
    P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
    P2="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
    P3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_BUSY_CYCLES"
    i=0
    for P in "$P1" "$P2" "$P3"; do
        i=$((i + 1))
        rm -rf "$R/gpurun_out/sqpmc_pairs_$i" "$R/gpurun_out/sqpmc_keys_$i"
        (cd /tmp && PL_ROUNDS=1 PL_REPS=1 TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv \
            -d "$R/gpurun_out/sqpmc_pairs_$i" -- "$R/dev/pairs_lab" 29 > "$R/gpurun_out/sqpmc_pairs_$i.log" 2>&1)
        stop_unless_ok $? "sqpmc pairs $i"
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/sqpmc_keys_$i" -- \
            python3 "$R/bench.py" --keys 536870912 --steps 1 --warmup 1 --no-cpu --no-e2e --no-vendor --configs "" \
            > "$R/gpurun_out/sqpmc_keys_$i.log" 2>&1)
        stop_unless_ok $? "sqpmc keys $i"
    done
    python3 dev/sqpmc.py gpurun_out
    ;;
sqc2)
    # SQ counters of the C2 sort (bench.py --keys 2^26 --k 4), three passes of <= 8 counters, against a C3
    # sort (2^29 keys, k = 8): is the k = 4 pass LDS-bound? (dev/sqpmc.py)
    P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
    P2="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
    P3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_BUSY_CYCLES"
    i=0
    for P in "$P1" "$P2" "$P3"; do
        i=$((i + 1))
        for cfg in "c2:--keys 67108864 --k 4" "keys:--keys 536870912"; do
            tag=${cfg%%:*}
            rm -rf "$R/gpurun_out/sqpmc_${tag}_$i"
            (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/sqpmc_${tag}_$i" -- \
                python3 "$R/bench.py" ${cfg#*:} --steps 1 --warmup 1 --no-cpu --no-e2e --no-vendor --configs "" \
                > "$R/gpurun_out/sqpmc_${tag}_$i.log" 2>&1)
            stop_unless_ok $? "sqc2 $tag $i"
        done
    done
    python3 dev/sqpmc.py gpurun_out c2,keys
    ;;
sqzipf)
    # SQ counters per dispatch of the Zipf-keys passes (bench.py --dist zipf, 2^29 keys), in issue order:
    # LDS address / bank conflicts of the clustered passes against the first (dev/sqpmc.py --order)
    P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
    rm -rf "$R/gpurun_out/sqzipf_keys_1"
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$R/gpurun_out/sqzipf_keys_1" -- \
        python3 "$R/bench.py" --keys 536870912 --dist zipf --steps 1 --warmup 1 --no-cpu --no-e2e --no-vendor --configs "" \
        > "$R/gpurun_out/sqzipf_keys_1.log" 2>&1)
    stop_unless_ok $? "sqzipf"
    python3 dev/sqpmc.py gpurun_out --order sqzipf_keys
    ;;
wgt)
    # per-workgroup durations of every scatter pass (dev/var_wgt.so: -DRSORT_WG_TIMES) and what the
    # slowest chunks of pass 1 hold: Zipf keys, Zipf pairs, uniform keys (dev/wgtimes_lab.py)
    cp cuda.radixsort_amd/librsort.so gpurun_out/wgt_lib.so
    cp dev/var_wgt.so cuda.radixsort_amd/librsort.so
    for args in "--dist zipf --dump gpurun_out/wgt_zipf_p1.csv" "--dist zipf --pass 2 --dump gpurun_out/wgt_zipf_p2.csv" \
                "--dist uniform"; do
        timeout -k 10 240 python dev/wgtimes_lab.py $args "$@" >> gpurun_out/wgt.log 2>&1
        rc=$?
        echo "[lab] wgt $args rc=$rc"
        [ $rc -eq 0 ] || break
    done
    cp gpurun_out/wgt_lib.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/wgt_lib.so
    cat gpurun_out/wgt.log
    ;;
c2tpc)
    # C2 (2^26 keys, k = 4) with tiles_per_chunk 16 (the plan's default: one resident wave of
    # workgroups), 8 and 4 (two and four waves: the dispatcher balances the later waves), raw next-digit
    # tables and tail scans (RSORT_NX_TAIL=1), alternating twice
    for rep in 1 2; do
        for tpc in ${C2_TPCS:-16 8 4}; do
            for tail in 0 1; do
                RSORT_LAB=1 RSORT_NX_TAIL=$tail timeout -k 10 120 python bench.py --keys 67108864 --k 4 --tiles-per-chunk $tpc \
                    --steps 20 --warmup 5 --no-cpu --no-vendor --no-e2e --configs "" > gpurun_out/c2tpc.json 2> gpurun_out/c2tpc.err
                stop_unless_ok $? "c2 tpc=$tpc tail=$tail" > /dev/null
                python3 - "$tpc" "$tail" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/c2tpc.json").read().strip().splitlines()[-1])
print("tpc %2s tail %s: %.4f ms/sort  scatter %.4f ms/pass  chunks %d  verified %s" % (sys.argv[1], sys.argv[2],
      d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["num_chunks"], d["verified"]))
PY
            done
        done
    done
    ;;
wgtk)
    # the same lab build: per-workgroup start / end of every pass of one sort (args: e.g. --k 4 --log2n 26)
    cp cuda.radixsort_amd/librsort.so gpurun_out/wgt_lib.so
    cp dev/var_wgt.so cuda.radixsort_amd/librsort.so
    timeout -k 10 240 python dev/wgtimes_lab.py --dist uniform "$@" >> gpurun_out/wgtk.log 2>&1
    rc=$?
    cp gpurun_out/wgt_lib.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/wgt_lib.so
    cat gpurun_out/wgtk.log
    stop_unless_ok $rc wgtk
    ;;
wgth)
    # the same lab build: per-workgroup durations of the joint-count histograms (Zipf, uniform keys;
    # WGT_VAR picks another lab build dev/var_$WGT_VAR.so, WGT_DISTS the distributions)
    cp cuda.radixsort_amd/librsort.so gpurun_out/wgt_lib.so
    cp dev/var_${WGT_VAR:-wgt}.so cuda.radixsort_amd/librsort.so
    echo "== ${WGT_VAR:-wgt}" >> gpurun_out/wgth.log
    for dist in ${WGT_DISTS:-zipf uniform}; do
        timeout -k 10 240 python dev/wgtimes_lab.py --dist $dist --hist "$@" >> gpurun_out/wgth.log 2>&1
        rc=$?
        echo "[lab] wgth $dist rc=$rc"
        [ $rc -eq 0 ] || break
    done
    cp gpurun_out/wgt_lib.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/wgt_lib.so
    cat gpurun_out/wgth.log
    ;;
ceiling)
    timeout -k 10 240 dev/ceiling_lab 30 10 > gpurun_out/ceiling.jsonl 2> gpurun_out/ceiling.err
    stop_unless_ok $? ceiling
    grep -v chunk_records gpurun_out/ceiling.jsonl | tail -n 30
    ;;
pfloor)
    # the pairs pass's write-stream floor (dev/ceiling_lab pairs, built here) and, on the same box, the
    # pairs kernel on uniform and Zipf pairs (bench.py, scatter ms per pass)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 dev/ceiling_lab.hip -o /tmp/ceiling_lab_p || exit 1
    timeout -k 10 120 /tmp/ceiling_lab_p 30 10 pairs > gpurun_out/pfloor.jsonl 2> gpurun_out/pfloor.err
    stop_unless_ok $? pfloor
    cat gpurun_out/pfloor.jsonl
    for d in uniform zipf; do
        timeout -k 10 200 python bench.py --dist $d --pairs --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e \
            --configs "" > gpurun_out/pfloor_$d.json 2> gpurun_out/pfloor_$d.err
        stop_unless_ok $? "pfloor $d"
        python3 - "$d" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/pfloor_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("pairs %-8s %8.3f ms/sort  scatter %.4f ms/pass (%.3f)  %s" % (sys.argv[1], d["ms_per_step"], r["avg_launch_ms"],
      r["frac"], d["verified"]))
PY
    done
    ;;
wgtx)
    cp cuda.radixsort_amd/librsort.so gpurun_out/wgt_lib.so
    cp dev/var_wgt.so cuda.radixsort_amd/librsort.so
    rc=0
    set -- "--dist uniform --log2n 30 --reps 4" "--dist uniform --log2n 26 --k 4 --reps 4" "--dist zipf --log2n 30 --reps 3"
    [ -n "$WGTX_ARGS" ] && set -- "$WGTX_ARGS"
    for args in "$@"; do
        timeout -k 10 240 python dev/wgtimes_lab.py $args >> gpurun_out/wgtx.log 2>&1
        rc=$?
        echo "[lab] wgtx $args rc=$rc"
        [ $rc -eq 0 ] || break
    done
    cp gpurun_out/wgt_lib.so cuda.radixsort_amd/librsort.so
    rm -f gpurun_out/wgt_lib.so
    cat gpurun_out/wgtx.log
    stop_unless_ok $rc wgtx
    ;;
cutw)
    : > gpurun_out/cutw.log
    for rep in 1 2; do
        for args in "--dist zipf --keys 268435456" "--dist zipf" "--dist zipf12" "--dist hot" "--dist zipf --pairs" \
                    "--dist hot --pairs"; do
            for w in 1 0; do
                if [ $w = 1 ]; then
                    timeout -k 10 200 python bench.py $args --steps 10 --warmup 3 --no-cpu --no-vendor --no-e2e --configs "" \
                        > gpurun_out/cutw.json 2> gpurun_out/cutw.err
                else
                    RSORT_LAB=1 RSORT_CUT_WEIGHTS=0 timeout -k 10 200 python bench.py $args --steps 10 --warmup 3 --no-cpu \
                        --no-vendor --no-e2e --configs "" > gpurun_out/cutw.json 2> gpurun_out/cutw.err
                fi
                stop_unless_ok $? "cutw $args w=$w" > /dev/null
                python3 - "$args" "$w" >> gpurun_out/cutw.log <<'PY'
import json, sys
d = json.loads(open("gpurun_out/cutw.json").read().strip().splitlines()[-1])
print("%-32s weights=%s %8.3f ms/sort  scatter %.4f ms/pass  hist %.3f  modes %s  %s" % (sys.argv[1], sys.argv[2],
      d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["phases_ms_per_step"]["histogram"],
      d["config"]["group_chunk_modes"], d["verified"]))
PY
            done
        done
    done
    cat gpurun_out/cutw.log
    ;;
prof)
    tag=$1
    shift
    bash profiles/run_profiles.sh "$tag" "$@"
    stop_unless_ok $? "prof $tag"
    ;;
pmc)
    C="TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_BUSY_avr TCC_EA0_WRREQ_STALL_sum"
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc $C -d "$R/gpurun_out/pmc_a" -o run -- \
        "$R/dev/scatter_lab" 30 "k8 1024x16 lines16" > "$R/gpurun_out/pmc_a.log" 2>&1) || exit $?
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc $C -d "$R/gpurun_out/pmc_b" -o run -- \
        "$R/dev/wc_lab" 30 > "$R/gpurun_out/pmc_b.log" 2>&1) || exit $?
    python3 dev/pmcdb.py gpurun_out/pmc_a gpurun_out/pmc_b
    ;;
dist)
    rm -rf "$R/gpurun_out/prof_dist"
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof_dist" -- python3 "$R/bench.py" --no-cpu --no-e2e --configs "" --dist-path \
        --steps 3 --warmup 1 "$@" > "$R/gpurun_out/prof_dist.log" 2>&1)
    stop_unless_ok $? dist
    tail -c 1500 "$R/gpurun_out/prof_dist.log"
    ;;
profiles)
    tag=$1
    bash profiles/run_profiles.sh "$tag" || exit $?
    bash profiles/run_profiles.sh "${tag}_zipf" --dist zipf || exit $?
    bash profiles/run_profiles.sh "${tag}_c4" --dist zipf --pairs || exit $?
    bash profiles/run_profiles.sh "${tag}_c2" --keys 67108864 --k 4 || exit $?
    for v in "" "--dist-full"; do
        d="$R/gpurun_out/prof_${tag}_dist${v:+_full}"
        rm -rf "$d"
        (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -- \
            python3 "$R/bench.py" --no-cpu --no-e2e --no-vendor --configs "" --dist-path $v --steps 3 --warmup 1 \
            > "$d.log" 2>&1)
        stop_unless_ok $? "dist $v"
        tail -c 600 "$d.log"
    done
    ;;
*)
    echo "unknown experiment: $exp (see the header of dev/lab.sh)"
    exit 2
    ;;
esac
