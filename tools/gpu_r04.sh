# round-4 GPU runner: `bash tools/gpu_r04.sh <step>...`; every step has its own
# time limit and the first failure ends the call (no retries)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
mkdir -p $O
for st in "$@"; do
  echo "== step $st $(date +%T)"
  case $st in
    tests)  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?
            grep -E "PASSED|FAILED|ERROR|SKIPPED" $O/tests.log | tail -4; tail -3 $O/tests.log; [ $rc = 0 ] || exit 1 ;;
    smoke)  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
            grep -v amdgpu.ids $O/smoke.log | tail -3 ;;
    bench)  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
            tail -1 $O/bench.json | cut -c1-900 ;;
    json4k) timeout -k 10 300 python bench.py --workload json4k --no-cpu > $O/json4k.json 2> $O/json4k.err || exit 1
            tail -1 $O/json4k.json | cut -c1-600 ;;
    dec)    timeout -k 10 400 python bench.py --mode decompress --no-cpu > $O/dec.json 2> $O/dec.err || exit 1
            tail -1 $O/dec.json | cut -c1-600 ;;
    mixed)  timeout -k 10 600 python bench.py --workload mixed16k --total 4194304 --steps 3 --no-cpu > $O/mixed.json 2> $O/mixed.err || exit 1
            tail -1 $O/mixed.json | cut -c1-600 ;;
    abslab) AB_SEED=0x5EED0003 timeout -k 10 600 python -u tools/ab_compress.py 2 65536 262144 3 gibson_amd/liblzf_hip.so gibson_amd/liblzf_hip_slab.so > $O/abslab.txt 2>&1 || exit 1
            cat $O/abslab.txt ;;
    k3t)    for L in timing slabtiming; do LZF_HIP_LIB=$PWD/gibson_amd/liblzf_hip_$L.so timeout -k 10 300 python -u tools/k3_timing.py 2 65536 262144 > $O/k3t_$L.txt 2>&1 || exit 1; echo $L; cat $O/k3t_$L.txt; done ;;
    ab:*)   # ab:<variant>[:<variant>] -- text64k configs[2] 256 K values, base vs variants (one process)
            v=${st#ab:}; libs="gibson_amd/liblzf_hip.so"; for x in ${v//:/ }; do libs="$libs gibson_amd/liblzf_hip_$x.so"; done
            AB_SEED=0x5EED0003 timeout -k 10 600 python -u tools/ab_compress.py 2 65536 262144 3 $libs > $O/ab_${v//:/_}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/ab_${v//:/_}.txt ;;
    env:*)  # env:<kind>:<n>:<count>:<setting>:<setting>... -- ab_env.py (settings use , and =)
            IFS=: read -r _ k nn c rest <<< "$st"; IFS=: read -ra sets <<< "$rest"
            timeout -k 10 600 python -u tools/ab_env.py $k $nn $c 3 "${sets[@]}" > $O/env_${k}_${nn}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/env_${k}_${nn}.txt ;;
    host)   for w in "2 65536 65536" "1 4096 524288" "3 16384 131072"; do set -- $w
              LZF_GPU_HOST_THREADS=16 timeout -k 10 400 python -u tools/host_path_bench.py $1 $2 $3 5 > $O/host_$1_$2.json 2> $O/host_$1_$2.err || exit 1
              cut -c1-400 $O/host_$1_$2.json; done ;;
    pmcmix) for c in FETCH_SIZE WRITE_SIZE; do
              timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d $O/pmc_mixed_$c -o run -- python3 bench.py --workload mixed16k --total 4194304 --steps 1 --warmup 0 --no-cpu > $O/pmc_mixed_$c.log 2>&1 || exit 1
              tail -1 $O/pmc_mixed_$c.log | cut -c1-200; done ;;
    dab:*)  # dab:<kind>:<n>:<count>:<variant>[:<variant>] -- decode A/B (AB_MODE=decompress), base vs variants
            IFS=: read -r _ k nn c rest <<< "$st"; libs="gibson_amd/liblzf_hip.so"; for x in ${rest//:/ }; do libs="$libs gibson_amd/liblzf_hip_$x.so"; done
            AB_MODE=decompress AB_SEED=$([ $k = 0 ] && echo 0x5EED0004 || ([ $k = 2 ] && echo 0x5EED0003 || ([ $k = 3 ] && echo 0x5EED0005 || echo 0x5EED0002))) \
              timeout -k 10 600 python -u tools/ab_compress.py $k $nn $c 5 $libs > $O/dab_${k}_${nn}_${rest//:/_}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/dab_${k}_${nn}_${rest//:/_}.txt ;;
    tokstat) timeout -k 10 300 python -u tools/dec_tstat.py 0 8192 1048576 gibson_amd/liblzf_hip_time.so gibson_amd/liblzf_hip_toktime.so > $O/tokstat.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/tokstat.txt ;;
    pmctok) timeout -k 10 600 bash tools/pmc_dec_ab.sh "" tok > $O/pmctok.txt 2>&1 || exit 1
            cat $O/pmctok.txt; cp gpurun_out/mix_*.txt $O/ ;;
    abk:*)  # abk:<kind>:<n>:<count>:<variant>[:<variant>] -- compress A/B, product vs variants
            IFS=: read -r _ k nn c rest <<< "$st"; libs="gibson_amd/liblzf_hip.so"; for x in ${rest//:/ }; do libs="$libs gibson_amd/liblzf_hip_$x.so"; done
            AB_SEED=$([ $k = 0 ] && echo 0x5EED0004 || ([ $k = 2 ] && echo 0x5EED0003 || ([ $k = 3 ] && echo 0x5EED0005 || echo 0x5EED0002))) \
              timeout -k 10 600 python -u tools/ab_compress.py $k $nn $c 3 $libs > $O/abk_${k}_${nn}_${rest//:/_}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/abk_${k}_${nn}_${rest//:/_}.txt ;;
    prof:*) # prof:<label>:<bench args, comma-separated> -- rocprofv3 kernel trace + stats of bench.py
            IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }
            timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$lab -o run -- python3 bench.py $args --no-cpu > $O/prof_$lab.log 2>&1 || exit 1
            python3 profiles/summarize.py $O/prof_$lab "bench.py $args (round 4)" > $O/kernel_stats_$lab.txt || exit 1
            rm -rf $O/prof_$lab; head -6 $O/kernel_stats_$lab.txt; grep '^{' $O/prof_$lab.log | tail -1 | cut -c1-300 ;;
    pmc:*)  # pmc:<label>:<bench args, comma-separated> -- FETCH_SIZE and WRITE_SIZE passes (one counter set per run)
            IFS=: read -r _ lab args <<< "$st"; args=${args//,/ }
            for c in FETCH_SIZE WRITE_SIZE; do
              timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${lab}_$c -o run -- python3 bench.py $args --no-cpu > $O/pmc_${lab}_$c.log 2>&1 || exit 1
              tail -1 $O/pmc_${lab}_$c.log | cut -c1-200; done ;;
    tstat:*) # tstat:<kind>:<n>:<count> -- pipe phase cycles (CD_TIMING build liblzf_hip_time.so)
            IFS=: read -r _ k nn c <<< "$st"
            timeout -k 10 300 python -u tools/dec_tstat.py $k $nn $c gibson_amd/liblzf_hip_time.so > $O/tstat_${k}_${nn}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/tstat_${k}_${nn}.txt ;;
    xo:*)   # xo:<kind>:<n>:<max count>:<counts, comma-separated> -- lane route vs window64 by batch size
            IFS=: read -r _ k nn c cs <<< "$st"
            XO_COUNTS=$cs timeout -k 10 600 python -u tools/crossover.py $k $nn $c > $O/xo_${k}_${nn}.txt 2>&1 || exit 1
            grep -v amdgpu.ids $O/xo_${k}_${nn}.txt ;;
    gpus2)  # the N-rank path rehearsed: two ranks on the one device, gloo barrier/reductions
            LZF_BENCH_BACKEND=gloo LZF_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/gpus2.json 2> $O/gpus2.err || exit 1
            tail -1 $O/gpus2.json | cut -c1-400
            LZF_BENCH_BACKEND=gloo LZF_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --mode decompress --total 4194304 --steps 2 --warmup 1 --no-cpu > $O/gpus2_dec.json 2> $O/gpus2_dec.err || exit 1
            tail -1 $O/gpus2_dec.json | cut -c1-400 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
