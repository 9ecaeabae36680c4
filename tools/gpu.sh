#!/bin/bash
# The one GPU-box driver (round 5; replaces the per-round and per-experiment
# scripts of rounds 1-4).  Run from the repo root on the box:
#     bash tools/gpu.sh [-o OUTDIR] STEP [STEP ...]
# Every step has its own time limit; the first failure ends the call (no
# retries, no further GPU step after a fault, abort or time limit).
#
# Steps
#   tests[:EXPR]        the -m gpu suite (pytest -k EXPR)
#   smoke               __graft_entry__.smoke()
#   bench[:ARGS]        bench.py line (ARGS comma-separated, e.g. bench:--workload,json4k)
#   benv:LABEL:ENV:ARGS bench.py ARGS under ENV (VAR=x,VAR2=y) -> bench_LABEL.json
#   prof:LABEL:ARGS     rocprofv3 --kernel-trace --stats of bench.py ARGS -> kernel_stats_LABEL.txt
#   pmc:LABEL:ARGS      FETCH_SIZE and WRITE_SIZE passes of bench.py ARGS (one counter per run)
#   mix:LABEL:ARGS      instruction-mix counter sets of bench.py ARGS (one set per run) -> mix_LABEL.txt
#   ab:K:N:C:V[:V..]    compress A/B in one process: product vs gibson_amd/liblzf_hip_V.so (tools/ab_compress.py)
#   dab:K:N:C:V[:V..]   the same for the decoder (AB_MODE=decompress)
#   env:K:N:C:S[:S..]   compress A/B of env settings (tools/ab_env.py; a setting uses , and =)
#   tstat:K:N:C         the pipe decoder's phase cycles (CD_TIMING build liblzf_hip_time.so)
#   kt:K:N:C:LIB        per-phase cycles of the table cand kernel (-DKT_TIMING build liblzf_hip_LIB.so)
#   ktr:K:N:C           per-step busy cycles of every cand wave (tools/kt_trace.py, liblzf_hip_ktlite.so)
#   k3:K:N:C:LIB        per-value counters of the record parse (-DKT_TIMING build liblzf_hip_LIB.so)
#   xo:K:N:C:COUNTS     routed generation vs window64 by batch size (tools/crossover.py)
#   host[:reg]          PCIe-inclusive host-path rates (tools/host_path_bench.py); :reg registered only
#   hostenv:LABEL:ENV:ARGS  tools/host_path_bench.py ARGS under ENV
#   hostsplit           registered text64k / json4k on LZF_GPU_DEVICES=0,0, round-robin vs block split
#   numa                registered text64k with the arenas bound to NUMA node 0, then node 1
#   trace:LABEL:ARGS    kernel + copy timeline of tools/host_path_bench.py ARGS (tools/trace_timeline.py)
#   gpus2               the N-rank bench path rehearsed with two ranks on the one device (gloo)
#   calib               FETCH_SIZE / WRITE_SIZE calibration (tools/fetch_calib.hip, built as tools/fetch_calib_bin)
#   pcie                tools/probe/pcie_probe.hip (built as tools/probe/pcie_probe_bin)
# K is the generator kind (0 Zipf text, 1 json, 2 sentence text, 3 mixed), N the
# value size, C the count; its BASELINE seed is picked from K.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/run
if [ "$1" = "-o" ]; then O=$2; shift 2; fi
mkdir -p "$O"
seed_of() { case $1 in 0) echo 0x5EED0004 ;; 2) echo 0x5EED0003 ;; 3) echo 0x5EED0005 ;; *) echo 0x5EED0002 ;; esac; }
libs_of() { local l="gibson_amd/liblzf_hip.so"; for x in ${1//:/ }; do l="$l gibson_amd/liblzf_hip_$x.so"; done; echo $l; }
quiet() { grep -v amdgpu.ids "$@"; }
for st in "$@"; do
  echo "== step $st $(date +%T)"
  case $st in
    tests|tests:*)
      k=${st#tests}; k=${k#:}
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread ${k:+-k "$k"} > $O/tests.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR|SKIPPED" $O/tests.log | tail -4; tail -3 $O/tests.log; [ $rc = 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
      quiet $O/smoke.log | tail -3 ;;
    bench|bench:*)
      a=${st#bench}; a=${a#:}; a=${a//,/ }; lab=$(echo "main$a" | tr -c 'a-zA-Z0-9\n' '_')
      timeout -k 10 600 python bench.py $a > $O/bench_$lab.json 2> $O/bench_$lab.err || exit 1
      tail -1 $O/bench_$lab.json | cut -c1-900 ;;
    benv:*)
      IFS=: read -r _ lab envs args <<< "$st"; args=${args//,/ }; envs=${envs//,/ }
      env $envs timeout -k 10 600 python bench.py $args > $O/bench_$lab.json 2> $O/bench_$lab.err || exit 1
      tail -1 $O/bench_$lab.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"].get("per_kernel_ms"), d["config"].get("roundtrip_ok"))' ;;
    prof:*)
      IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$lab -o run -- python3 bench.py $args --no-cpu > $O/prof_$lab.log 2>&1 || exit 1
      python3 profiles/summarize.py $O/prof_$lab "bench.py $args" > $O/kernel_stats_$lab.txt || exit 1
      rm -rf $O/prof_$lab; head -8 $O/kernel_stats_$lab.txt; grep '^{' $O/prof_$lab.log | tail -1 | cut -c1-300 ;;
    pmc:*)
      IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${lab}_$c -o run -- python3 bench.py $args --no-cpu --steps 1 --warmup 0 > $O/pmc_${lab}_$c.log 2>&1 || exit 1
        tail -1 $O/pmc_${lab}_$c.log | cut -c1-200; done ;;
    mix:*)
      IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }; i=0
      for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
                 "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/mix_$lab/p$i -o run -- python3 bench.py $args --no-cpu --steps 1 --warmup 0 > $O/mix_$lab.p$i.log 2>&1 || exit 1
      done
      python3 tools/pmc_table.py $O/mix_$lab/p1 $O/mix_$lab/p2 $O/mix_$lab/p3 > $O/mix_$lab.txt || exit 1
      grep lzf_ $O/mix_$lab.txt ;;
    ab:*|dab:*)
      IFS=: read -r kindab k nn c rest <<< "$st"
      mode=compress; [ $kindab = dab ] && mode=decompress
      AB_MODE=$mode AB_SEED=$(seed_of $k) timeout -k 10 600 python -u tools/ab_compress.py $k $nn $c $([ $mode = decompress ] && echo 5 || echo 3) $(libs_of "$rest") > $O/${kindab}_${k}_${nn}_${rest//:/_}.txt 2>&1 || exit 1
      quiet $O/${kindab}_${k}_${nn}_${rest//:/_}.txt ;;
    env:*)
      IFS=: read -r _ k nn c rest <<< "$st"; IFS=: read -ra sets <<< "$rest"
      timeout -k 10 600 python -u tools/ab_env.py $k $nn $c 3 "${sets[@]}" > $O/env_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/env_${k}_${nn}.txt ;;
    tstat:*)
      IFS=: read -r _ k nn c <<< "$st"
      timeout -k 10 300 python -u tools/dec_tstat.py $k $nn $c gibson_amd/liblzf_hip.so gibson_amd/liblzf_hip_time.so > $O/tstat_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/tstat_${k}_${nn}.txt ;;
    kt:*)
      # kt:K:N:C:LIB -- per-phase cycles of the table cand kernel (a -DKT_TIMING build gibson_amd/liblzf_hip_LIB.so)
      IFS=: read -r _ k nn c lib <<< "$st"
      LZF_HIP_LIB=$PWD/gibson_amd/liblzf_hip_$lib.so timeout -k 10 300 python -u tools/kt_timing.py $k $nn $c > $O/kt_${lib}_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/kt_${lib}_${k}_${nn}.txt ;;
    ktr:*)
      # ktr:K:N:C -- per-step busy cycles of every cand wave (-DKT_TIMING -DKT_LITE build liblzf_hip_ktlite.so)
      IFS=: read -r _ k nn c <<< "$st"
      timeout -k 10 300 python -u tools/kt_trace.py $k $nn $c > $O/ktr_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/ktr_${k}_${nn}.txt ;;
    k3:*)
      # k3:K:N:C:LIB -- per-value counters of the record parse (a -DKT_TIMING build gibson_amd/liblzf_hip_LIB.so)
      IFS=: read -r _ k nn c lib <<< "$st"
      LZF_HIP_LIB=$PWD/gibson_amd/liblzf_hip_$lib.so timeout -k 10 300 python -u tools/k3_timing.py $k $nn $c > $O/k3_${lib}_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/k3_${lib}_${k}_${nn}.txt ;;
    xo:*)
      IFS=: read -r _ k nn c cs <<< "$st"
      XO_COUNTS=$cs timeout -k 10 600 python -u tools/crossover.py $k $nn $c > $O/xo_${k}_${nn}.txt 2>&1 || exit 1
      quiet $O/xo_${k}_${nn}.txt ;;
    host|host:reg)
      for w in "2 65536 65536 text64k" "1 4096 524288 json4k" "3 16384 131072 mixed16k"; do set -- $w
        if [ $st = host ]; then
          LZF_GPU_HOST_THREADS=16 timeout -k 10 300 python tools/host_path_bench.py $1 $2 $3 5 > $O/host_$4_staged.json 2> $O/host_$4_staged.err || exit 1
          timeout -k 10 300 python tools/host_path_bench.py $1 $2 $3 5 --register --devices 0,0 > $O/host_$4_reg_dev00.json 2> $O/host_$4_reg_dev00.err || exit 1
        fi
        timeout -k 10 300 python tools/host_path_bench.py $1 $2 $3 5 --register > $O/host_$4_reg.json 2> $O/host_$4_reg.err || exit 1
        cut -c1-300 $O/host_$4_reg.json; done ;;
    hostsplit)
      # round 6: the library's two splits over two workers on the one device
      # (LZF_GPU_DEVICES=0,0), registered arenas, text64k and json4k
      for w in "2 65536 65536 text64k" "1 4096 524288 json4k"; do set -- $w
        for sp in rr block; do
          LZF_GPU_SPLIT=$sp timeout -k 10 300 python tools/host_path_bench.py $1 $2 $3 5 --register --devices 0,0 > $O/host_$4_reg_dev00_$sp.json 2> $O/host_$4_reg_dev00_$sp.err || exit 1
          python3 -c "import json;d=json.load(open('$O/host_$4_reg_dev00_$sp.json'));print('$4 $sp', d['split'], d['compress_GBps'], d['decompress_GBps'], d['roundtrip_GBps'], d['roundtrip_ok'])"
        done; done ;;
    numa)
      # round 6: registered arenas placed on each NUMA node (the GPU sits on
      # node 0): what a worker pays for an arena across the socket link
      for node in 0 1; do
        timeout -k 10 300 python tools/host_path_bench.py 2 65536 65536 5 --register --arena-node $node > $O/host_text64k_reg_node$node.json 2> $O/host_text64k_reg_node$node.err || { tail -3 $O/host_text64k_reg_node$node.err; exit 1; }
        python3 -c "import json;d=json.load(open('$O/host_text64k_reg_node$node.json'));print('node $node', d['arena_node'], d['compress_GBps'], d['decompress_GBps'], d['roundtrip_GBps'], d['roundtrip_ok'])"
      done ;;
    hostenv:*)
      # hostenv:LABEL:ENV:ARGS -- tools/host_path_bench.py ARGS under ENV (VAR=x,VAR2=y)
      IFS=: read -r _ lab envs args <<< "$st"; args=${args//,/ }; envs=${envs//,/ }
      env $envs timeout -k 10 300 python tools/host_path_bench.py $args > $O/host_$lab.json 2> $O/host_$lab.err || exit 1
      python3 -c "import json;d=json.load(open('$O/host_$lab.json'));print('$lab', d['compress_GBps'], d['decompress_GBps'], d['roundtrip_GBps'], d['roundtrip_ok'])" ;;
    trace:*)
      IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_$lab -o run -- python3 tools/host_path_bench.py $args > $O/trace_$lab.log 2>&1 || exit 1
      python3 tools/trace_timeline.py $O/trace_$lab run > $O/timeline_$lab.txt || exit 1
      wc -l $O/timeline_$lab.txt ;;
    gpus2)
      LZF_BENCH_BACKEND=gloo LZF_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/gpus2.json 2> $O/gpus2.err || exit 1
      tail -1 $O/gpus2.json | cut -c1-400 ;;
    calib)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/calib_$c -o run -- ./tools/fetch_calib_bin > $O/calib_$c.log 2>&1 || exit 1
      done
      timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/calib_trace -o run -- ./tools/fetch_calib_bin > $O/calib_trace.log 2>&1 || exit 1 ;;
    pcie)
      timeout -k 10 120 ./tools/probe/pcie_probe_bin 1024 65536 > $O/pcie_64k.json || exit 1
      timeout -k 10 120 ./tools/probe/pcie_probe_bin 1024 4096 > $O/pcie_4k.json || exit 1
      cat $O/pcie_64k.json $O/pcie_4k.json ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
