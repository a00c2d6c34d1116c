#!/bin/bash
# One gpurun call made of named steps (replaces the per-call rNNx.sh launch lines).
# Every GPU step runs under its own time limit; the chain stops at the first step
# that fails (a failing test run stops it too, unless the step is marked "tests?").
#
# usage: tools_dev/gpu_session.sh TAG STEP [STEP ...]
#   tests[=LIB]          pytest -m gpu (LIB: an ab_libs/NAME.so to load instead)
#   tests?[=LIB]         the same, but a test failure (pytest rc 1) does not stop the chain
#   bench                the default bench.py line -> TAG_bench.json
#   ab=N:LIB[,LIB...]    alternating bench A/B: default library vs each ab_libs/LIB.so, N rounds
#   ops=MODE:B[:LIB[:K=V]]  per-op dispatch intervals + wave spans (tools_dev/mode_ops.py);
#                        LIB "-" = the default library; K=V e.g. MODE_XA=direct, MODE_KV=bf16
#   tl=MODE:B[:OPS[:LIB]]  in-kernel phase timeline (tools_dev/diag_timeline.py, PHASES=1); OPS comma-separated
#   prof[=K=V]           rocprofv3 kernel-trace summary of the bench (eager) + phase cut (K=V: env of the run)
#   pmc                  PMC passes (tools_dev/pmc_collect.sh TAG)
#   codec[=LIB[:K=V]]    codec wall / device time per call (tools_dev/codec_latency.py); LIB "-" = default
#   cprof[=LIB]          rocprofv3 kernel trace of 3 codec decodes, per-dispatch table of the last
#   cpmc[=LIB]           the codec's SQ / TCC / TCP counter passes (tools_dev/codec_pmc.sh)
#   ctl[=LIB]            the residual-block kernel's phase stamps per stage (tools_dev/codec_rb_timeline.py)
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for STEP in "$@"; do
  name=${STEP%%=*}; arg=${STEP#*=}; [ "$arg" = "$STEP" ] && arg=""
  case "$name" in
    tests|tests\?)
      env=()
      [ -n "$arg" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$arg.so")
      log="$OUT/${TAG}_tests${arg:+_$arg}.log"
      set +e
      env "${env[@]}" timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > "$log" 2>&1
      rc=$?
      set -e
      tail -1 "$log"
      if [ $rc -ne 0 ]; then
        if [ "$name" = "tests?" ] && [ $rc -eq 1 ]; then echo "tests failed (continuing)"; else echo "tests rc=$rc"; exit $rc; fi
      fi ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$OUT/${TAG}_bench.log" 2>&1
      tail -1 "$OUT/${TAG}_bench.log" > "$OUT/${TAG}_bench.json"
      echo "bench ok" ;;
    ab)
      n=${arg%%:*}; libs=${arg#*:}
      bash tools_dev/ab_lib.sh "${TAG}_ab" "$n" $(echo "$libs" | tr ',' '\n' | sed 's#^#ab_libs/#; s#$#.so#') > "$OUT/${TAG}_ab.txt" 2>&1
      cat "$OUT/${TAG}_ab.txt" ;;
    ops)
      IFS=: read -r mode b lib kv <<< "$arg"
      env=()
      [ -n "$lib" ] && [ "$lib" != "-" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$lib.so")
      [ "$lib" = "-" ] && lib=""
      suf="${lib:+_$lib}${kv:+_${kv//=/-}}"
      env "${env[@]}" timeout -k 10 200 python -u tools_dev/mode_ops.py "$mode" "$b" $kv > "$OUT/${TAG}_ops_${mode}_b${b}${suf}.txt" 2>&1
      head -1 "$OUT/${TAG}_ops_${mode}_b${b}${suf}.txt" ;;
    tl)
      IFS=: read -r mode b ops lib <<< "$arg"
      env=()
      [ -n "$lib" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$lib.so")
      env "${env[@]}" PHASES=1 timeout -k 10 200 python -u tools_dev/diag_timeline.py "$mode" "$b" $(echo "$ops" | tr ',' ' ') \
        > "$OUT/${TAG}_tl_${mode}_b${b}${lib:+_$lib}.txt" 2>&1
      echo "timeline ok" ;;
    prof)
      # arg (optional): K=V set for the profiled run, e.g. prof=MAGPIE_STREAM_PRIO=0
      d="$OUT/${TAG}_prof${arg:+_${arg//=/-}}"
      env MAGPIE_EAGER=1 $arg timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$d" -o prof \
        -- python3 -u bench.py --no-cpu-baseline --no-extra > "$d.bench.log" 2>&1
      python3 tools_dev/prof_phase.py "$d/prof_kernel_trace.csv" "$d/phase_kernel_stats.csv" > "$d.phase.log"
      echo "rocprof ${arg:-default}: $(head -1 "$d.phase.log")" ;;
    pmc)
      bash tools_dev/pmc_collect.sh "$TAG" > "$OUT/${TAG}_pmc.log" 2>&1
      echo "pmc ok" ;;
    codec)
      IFS=: read -r lib kv <<< "$arg"
      env=()
      [ -n "$lib" ] && [ "$lib" != "-" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$lib.so")
      [ "$lib" = "-" ] && lib=""
      [ -n "$kv" ] && env+=("$kv")
      suf="${lib:+_$lib}${kv:+_${kv//=/-}}"
      env "${env[@]}" timeout -k 10 200 python -u tools_dev/codec_latency.py > "$OUT/${TAG}_codec${suf}.txt" 2>&1
      echo "codec ${lib:-default} ${kv}: $(tail -1 "$OUT/${TAG}_codec${suf}.txt")" ;;
    cprof)
      env=()
      [ -n "$arg" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$arg.so")
      d="$OUT/${TAG}_cprof${arg:+_$arg}"
      MAGPIE_LIB="${env[0]#MAGPIE_LIB=}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$d" -o prof \
        -- python3 -u tools_dev/codec_prof.py > "$d.log" 2>&1
      python3 tools_dev/codec_trace_report.py "$d/prof_kernel_trace.csv" > "$d.txt"
      tail -12 "$d.txt" ;;
    cpmc)
      MAGPIE_LIB="${arg:+$PWD/ab_libs/$arg.so}" bash tools_dev/codec_pmc.sh > "$OUT/${TAG}_cpmc${arg:+_$arg}.log" 2>&1
      cp gpurun_out/cpmc/report.txt "$OUT/${TAG}_cpmc${arg:+_$arg}.txt"
      echo "codec pmc ok" ;;
    ctl)
      env=()
      [ -n "$arg" ] && env=(MAGPIE_LIB="$PWD/ab_libs/$arg.so")
      env "${env[@]}" timeout -k 10 200 python -u tools_dev/codec_rb_timeline.py > "$OUT/${TAG}_ctl${arg:+_$arg}.txt" 2>&1
      cat "$OUT/${TAG}_ctl${arg:+_$arg}.txt" ;;
    abkv)
      # alternating env A/B, f32 B=1: abkv=N:K=V[,K=V...]|K=V...   ('|' separates the settings)
      n=${arg%%:*}; rest=${arg#*:}
      IFS='|' read -r -a sets <<< "$rest"
      for k in "${!sets[@]}"; do sets[$k]=$(echo "${sets[$k]}" | tr ',' ' '); done
      bash tools_dev/ab_kv.sh "${TAG}_abkv" "$n" "${sets[@]}" > "$OUT/${TAG}_abkv.txt" 2>&1
      cat "$OUT/${TAG}_abkv.txt" ;;
    e2e)
      # configs[2] end to end under codec background CU shares: e2e=CUS,CUS:ROUNDS
      IFS=: read -r cus rounds <<< "${arg:-0,64:2}"
      timeout -k 10 400 python -u tools_dev/e2e_ab.py "$cus" "${rounds:-2}" > "$OUT/${TAG}_e2e.txt" 2>&1
      cat "$OUT/${TAG}_e2e.txt" ;;
    pre)
      # per-kernel time of one preamble (tools_dev/preamble_prof.py); arg: weights:B:T[:LIB]
      IFS=: read -r w b t lib <<< "${arg:-f32:1:64}"
      d="$OUT/${TAG}_pre_${w}_b${b}${lib:+_$lib}"
      MAGPIE_EAGER=0 MAGPIE_LIB="${lib:+$PWD/ab_libs/$lib.so}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$d" -o prof \
        -- python3 -u tools_dev/preamble_prof.py "$w" "$b" "$t" 3 > "$d.log" 2>&1
      python3 tools_dev/preamble_report.py "$d/prof_kernel_trace.csv" 3 > "$d.txt"
      head -1 "$d.txt"; grep "wall ms" "$d.log" ;;
    prewall)
      # preamble wall time without the profiler: arg weights:B:T[:LIB[:K=V]]
      IFS=: read -r w b t lib kv <<< "${arg:-f32:1:64}"
      echo -n "[$lib $kv] "
      env MAGPIE_LIB="${lib:+$PWD/ab_libs/$lib.so}" $kv timeout -k 10 200 python3 -u tools_dev/preamble_prof.py "$w" "$b" "$t" 10 ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "session $TAG done"
