#!/bin/bash
# One parameterised GPU-box script (replaces round 3's 45 per-call scripts):
#   gpurun --timeout 1200 -- bash tools/gpu/lease.sh <tag> <step>...
# Steps run in order, each under its own time limit, output to gpurun_out/<tag>/;
# the first failing step ends the call (no GPU step after a failure or a timeout).
#   tests            the whole -m gpu suite
#   tests:<files>    -m gpu on the comma-separated test files
#   smoke            __graft_entry__.smoke()
#   bench            the driver's command (bench.py --gpus 1 --steps 20 --warmup 5)
#   bench:<cfg>      bench.py --config <cfg> (C1..C5, NS) at its usual length
#   bench1000        the default 1000-step C2 bench
#   benchr:<cfg>     bench.py --config <cfg> --init random (a developed field)
#   prof:<cfg>       profiles/collect.sh (kernel trace + FETCH/WRITE passes) of bench --config <cfg>
#   tier             tools/tier_pattern_bench 16 and 32 (the C2 decision gate)
#   tierbench        the C2 bench through the two-tier launches (STENCIL_TK_TIER=1, debug library)
#   ramp             tools/ramp_probe.py under a rocprofv3 kernel trace (per-launch durations by phase)
#   sq:<cfg>         profiles/collect_sq.sh (SQ / LDS / TCC counter passes) of bench --config <cfg>
#   nstrace          three separate NS bench processes, each under a kernel trace (per-launch durations per process)
#   fastab           tools/ab.py at 512^3: the interior fast path as shipped vs on every tile (timing only) vs off
#   libab:<t1,t2..>  (LIBAB_FP32_ONLY=1: fp32 shapes only) tools/time_lib.py on build/variants/lib_<t>.so (tools/lib_variants.sh), one process per run,
#                    alternating the variants, 3 rounds over C2 / 2048^2 x 512 / NS / fp32 4096^2 x 256
#   libdigest:<t,..> tools/lib_digest.py per variant and the product library (bitwise check of variants)
#   libabbox:<t,..>  the same over box shapes: C5 2048^3 / 2048^2 x 256 / 512^3 fp64
#   rankof:<cfg>:<N>[:nosig] bench.py --config <cfg> --rank-of N --exchange loopback: one interior rank of the N-GPU job
#   plain:<star|box>:<dt>:nx:ny:nz:sweeps  tools/time_lib.py on the product library (one grid, AUTO)
#   zcab             tools/ab.py on 4096^2 x 512 fp64: z-chunk lengths (STENCIL_TK_ZCHUNK) of the wide-plane strip launch
#   padscan:nx:ny:nz:sweeps[:dtype[:pad,pad..]]  tools/time_lib.py (debug library) over STENCIL_ROW_PAD values
#   loop:<cfg>       bench.py --config <cfg> --exchange loopback (the whole grid as one periodic slab: an interior rank)
#   slabgap          tools/slab_gap.py: one K = 4 launch plain / slab layout / halo flags / signalled / slab job
#   c1ab             tools/c1_ab.py: the C1 region variants (branch-free ghost selects) interleaved, fp64 + fp32
#   xr:<cfg>:<N>:<ex>:<var>[:trace]  bench.py --rank-of N (0: none) --exchange loopback|nccl-self with the round
#                    variant ovl | serial | xcu<C>[x] (STENCIL_SLAB_XCU[_EXCL]), optionally under a kernel trace
#   c1probe          tools/c1_probe.py (C1 wall vs device time, eager vs one graph), then under a kernel trace
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
n=0
for step in "$@"; do
  echo "[lease] $TAG: $step $(date +%T)"
  case "$step" in
    tests) timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
             > "$O/gpu_tests.txt" 2>&1 ;;
    tests:*) n=$((n + 1))
             timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
             $(echo "${step#tests:}" | tr ',' ' ') > "$O/gpu_tests_part$n.txt" 2>&1 ;;
    testk:*) IFS=':' read -r tf te <<< "${step#testk:}"   # testk:<file>:<-k expression>
             n=$((n + 1))
             timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$tf" -k "$te" \
               > "$O/gpu_tests_k$n.txt" 2>&1 ;;
    smoke) timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench) f="$O/bench_driver.json"; k2=1; while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/bench_driver_$k2.json"; done
           timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$f" 2>> "$O/bench.err" ;;
    bench1000) f="$O/bench_1000.json"; k2=1; while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/bench_1000_$k2.json"; done
             timeout -k 10 200 python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline > "$f" 2>> "$O/bench.err" ;;
    bench:*) c=${step#bench:}
             case "$c" in C1) a="--steps 100 --warmup 10";; C5) a="--steps 32 --warmup 4";; *) a="--steps 40 --warmup 4";; esac
             timeout -k 10 400 python3 bench.py --config "$c" $a > "$O/bench_$c.json" 2>> "$O/bench.err" ;;
    benchr:*) c=${step#benchr:}   # the same on a developed field (uniform random interior)
             case "$c" in C1) a="--steps 100 --warmup 10";; C5) a="--steps 32 --warmup 4";; *) a="--steps 40 --warmup 4";; esac
             timeout -k 10 400 python3 bench.py --config "$c" --init random $a --no-cpu-baseline \
               > "$O/bench_${c}_random.json" 2>> "$O/bench.err" ;;
    prof:*) c=${step#prof:}
            case "$c" in C5) a="--steps 8 --warmup 0";; *) a="--steps 100 --warmup 5";; esac
            bash profiles/collect.sh "${TAG}_$c" --config "$c" $a --no-cpu-baseline > "$O/collect_$c.log" 2>&1 ;;
    proflong:*) c=${step#proflong:}   # the same at 1000 sweeps (one call: the long-job work orders)
            bash profiles/collect.sh "${TAG}_${c}long" --config "$c" --steps 1000 --warmup 20 --no-cpu-baseline \
              > "$O/collect_${c}long.log" 2>&1 ;;
    sq:*) c=${step#sq:}
          case "$c" in C1) a="--steps 100 --warmup 10";; C5) a="--steps 8 --warmup 0";; *) a="--steps 40 --warmup 4";; esac
          PROG=bench.py bash profiles/collect_sq.sh "${TAG}_$c" --config "$c" $a --no-cpu-baseline > "$O/sq_$c.log" 2>&1 ;;
    tier) timeout -k 10 120 tools/tier_pattern_bench 16 > "$O/tier16.txt" 2>&1 &&
          timeout -k 10 120 tools/tier_pattern_bench 32 > "$O/tier32.txt" 2>&1 ;;
    ramp) (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/ramp" -o run -- \
             python3 "$R/tools/ramp_probe.py" > "$O/ramp.log" 2>&1) ;;
    nstrace) for i in 1 2 3; do
               (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/nstrace$i" \
                 -o run -- python3 "$R/bench.py" --config NS --steps 40 --warmup 4 --no-cpu-baseline \
                 > "$O/nstrace$i.json" 2>> "$O/bench.err") || exit 1
             done ;;
    fastab) timeout -k 10 180 python3 tools/ab.py --grid 512 512 512 --steps 4 --reps 9 --launches 10 \
              --variant STENCIL_TK_FAST=1 --variant STENCIL_TK_FAST=2,NOCHECK=1 --variant STENCIL_TK_FAST=0 \
              > "$O/fast_ab.txt" 2>&1 ;;
    libab:*) IFS=',' read -r -a tags <<< "${step#libab:}"
             for rep in 1 2 3; do
               shapes=("star fp64 512 512 512 1000 2" "star fp64 2048 2048 512 200 2" "star fp64 2048 2048 2048 40 2"
                       "star fp32 4096 4096 256 200 2")
               [ -n "${LIBAB_FP32_ONLY:-}" ] && shapes=("star fp32 4096 4096 256 200 2" "star fp32 2048 2048 512 200 2")
               for shp in "${shapes[@]}"; do
                 for t in "${tags[@]}"; do
                   # shellcheck disable=SC2086
                   timeout -k 10 120 python3 tools/time_lib.py "build/variants/lib_$t.so" $shp >> "$O/lib_ab.txt" 2>> "$O/lib_ab.err" \
                     || exit 1
                 done
               done
             done ;;
    libdigest:*) # libdigest:<t1,t2..> -- tools/lib_digest.py per variant (and the product library): equal digests per
          # shape = bitwise equal results; odd nx (partial fp32 lane pairs), big / small planes, fp32 and fp64
          IFS=',' read -r -a tags <<< "${step#libdigest:}"
          for shp in "star fp32 4096 4096 64 23" "star fp32 1031 517 40 13" "star fp32 300 250 40 7" \
                     "star fp32 2049 1023 96 11" "star fp64 512 512 512 9" "star fp64 2048 2048 64 9" "star fp64 301 257 33 6"; do
            for t in product "${tags[@]}"; do
              lib="build/variants/lib_$t.so"; [ "$t" = product ] && lib=stencil_amd/libstencil_hip.so
              # shellcheck disable=SC2086
              timeout -k 10 120 python3 tools/lib_digest.py "$lib" $shp | sed "s/^/$t: /" >> "$O/lib_digest.txt" \
                2>> "$O/lib_ab.err" || exit 1
            done
          done ;;
    libabbox:*) IFS=',' read -r -a tags <<< "${step#libabbox:}"
             for rep in 1 2 3; do
               for shp in "box fp64 2048 2048 2048 16 2" "box fp64 2048 2048 256 40 2" "box fp64 512 512 512 200 2"; do
                 for t in "${tags[@]}"; do
                   # shellcheck disable=SC2086
                   timeout -k 10 120 python3 tools/time_lib.py "build/variants/lib_$t.so" $shp >> "$O/lib_ab_box.txt" \
                     2>> "$O/lib_ab.err" || exit 1
                 done
               done
             done ;;
    rankof:*) IFS=':' read -r c nr ns <<< "${step#rankof:}"
             case "$c" in C5) a="--steps 16 --warmup 4";; *) a="--steps 40 --warmup 4";; esac
             [ "$ns" = nosig ] && a="$a --no-signal"
             timeout -k 10 400 python3 bench.py --config "$c" --rank-of "$nr" --exchange loopback $a --no-cpu-baseline \
               > "$O/bench_${c}_rank_of_$nr${ns:+_$ns}.json" 2>> "$O/bench.err" ;;
    plain:*) IFS=':' read -r shp dt nx ny nz sw <<< "${step#plain:}"   # the single-grid kernel rate of one shape
             timeout -k 10 300 python3 tools/time_lib.py stencil_amd/libstencil_hip.so "$shp" "$dt" "$nx" "$ny" "$nz" "$sw" 3 \
               >> "$O/plain.txt" 2>> "$O/bench.err" ;;
    zcab) STENCIL_TK_VERBOSE=1 timeout -k 10 300 python3 tools/ab.py --grid 4096 4096 512 --steps 4 --reps 5 --launches 3 \
              --variant STENCIL_TK_ZCHUNK=0 --variant STENCIL_TK_ZCHUNK=256 --variant STENCIL_TK_ZCHUNK=128 \
              --variant STENCIL_TK_ZCHUNK=64 --variant STENCIL_TK_ZCHUNK=32 > "$O/zc_ab.txt" 2>&1 ;;
    padscan:*) IFS=':' read -r nx ny nz sw dt pads <<< "${step#padscan:}"
             dt=${dt:-fp64}; pads=${pads:-0,16,32,64,128,256,512,1024}
             for rep in 1 2; do
               for pad in ${pads//,/ }; do
                 STENCIL_ROW_PAD=$pad timeout -k 10 200 python3 tools/time_lib.py stencil_amd/libstencil_hip_debug.so star "$dt" \
                   "$nx" "$ny" "$nz" "$sw" 2 | sed "s/^/pad $pad: /" >> "$O/padscan.txt" 2>> "$O/bench.err" || exit 1
               done
             done ;;
    pitchscan:*) # pitchscan:<dtype>:<cells per plane>:<nz>:<sweeps>:<w1,w2,..> -- row-pitch scan over plane widths: each
          # width raw (STENCIL_ROW_RULE=0), +128 B, +2 KiB, and as the product pads it; ny = cells / width
          IFS=':' read -r dt cells nz sw widths <<< "${step#pitchscan:}"
          es=8; [ "$dt" = fp32 ] && es=4
          for rep in 1 2; do
            for w in ${widths//,/ }; do
              ny=$((cells / w))
              for v in "STENCIL_ROW_RULE=0:0" "STENCIL_ROW_RULE=0:$((128 / es))" "STENCIL_ROW_RULE=0:$((2048 / es))" "STENCIL_ROW_RULE=1:0"; do
                env "${v%%:*}" STENCIL_ROW_PAD="${v##*:}" timeout -k 10 200 python3 tools/time_lib.py \
                  stencil_amd/libstencil_hip_debug.so star "$dt" "$w" "$ny" "$nz" "$sw" 2 \
                  | sed "s/^/${v%%:*} pad ${v##*:}: /" >> "$O/pitchscan_$dt.txt" 2>> "$O/bench.err" || exit 1
              done
            done
          done ;;
    loop:*) c=${step#loop:}
            timeout -k 10 300 python3 bench.py --config "$c" --exchange loopback --steps 40 --warmup 4 --no-cpu-baseline \
              > "$O/bench_${c}_loopback.json" 2>> "$O/bench.err" ;;
    slabgap) timeout -k 10 300 python3 tools/slab_gap.py 4096 4096 512 > "$O/slab_gap.txt" 2>&1 &&
             timeout -k 10 300 python3 tools/slab_gap.py 512 512 512 >> "$O/slab_gap.txt" 2>&1 ;;
    slabtrace) (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/slabtrace" -o run -- \
                 python3 "$R/tools/slab_gap.py" 512 512 512 --reps 3 > "$O/slabtrace.log" 2>&1) ;;
    slabgapnp) STENCIL_SLAB_NOPRIO=1 timeout -k 10 300 python3 tools/slab_gap.py 4096 4096 512 > "$O/slab_gap_noprio.txt" 2>&1 &&
             STENCIL_SLAB_NOPRIO=1 timeout -k 10 300 python3 tools/slab_gap.py 512 512 512 >> "$O/slab_gap_noprio.txt" 2>&1 ;;
    c1ab) timeout -k 10 120 python3 tools/c1_ab.py --dtype fp64 --variant 0 --variant 92416 > "$O/c1_ab.txt" 2>&1 &&
          timeout -k 10 120 python3 tools/c1_ab.py --dtype fp64 --order dma --variant 0 --variant 92416 >> "$O/c1_ab.txt" 2>&1 &&
          timeout -k 10 120 python3 tools/c1_ab.py --dtype fp32 --variant 0 --variant 92808 >> "$O/c1_ab.txt" 2>&1 ;;
    c1probe) timeout -k 10 120 python3 tools/c1_probe.py > "$O/c1_probe.txt" 2>&1 &&
             (cd /tmp && TMPDIR=/tmp timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/c1trace" \
               -o run -- python3 "$R/tools/c1_probe.py" --reps 10 > "$O/c1_probe_traced.txt" 2>&1) ;;
    xr:*) # xr:<cfg>:<N>:<exchange>:<variant>[:trace] -- round-5 rehearsal matrix: one interior rank of the
          # N-GPU job (N = 0: the config's whole grid as one periodic slab) with loopback / nccl-self halos;
          # variant ovl (default rounds) | serial | xcu<C> | xcu<C>x (exchange on C CUs per XCD, x: launches off them)
          IFS=':' read -r c nr ex var tr <<< "${step#xr:}"
          envs=()
          for v in ${var//+/ }; do   # variants combine with '+', e.g. nosig+xcu1x
            case "$v" in
              ovl) ;; serial) envs+=(STENCIL_SLAB_SERIAL=1) ;; rser) envs+=(STENCIL_SLAB_ROLLING_OVERLAP=0) ;;
              nosig) envs+=(STENCIL_SLAB_SIGNAL=0) ;; cpwait) envs+=(STENCIL_SLAB_CPWAIT=1) ;;
              wire*) envs+=(STENCIL_SLAB_WIRE_GBPS=${v#wire}) ;;   # emulated xGMI wire time (debug library)
              nox) envs+=(STENCIL_SLAB_XCU=0) ;; noexcl) envs+=(STENCIL_SLAB_XCU_EXCL=0) ;;
              nostage) envs+=(STENCIL_SLAB_STAGED=0) ;; spare*) envs+=(STENCIL_TK_SIG_SPARE=${v#spare}) ;;
              nogate) envs+=(STENCIL_SLAB_GATE=0) ;; packxcd*) envs+=(STENCIL_TK_PACK_XCD=${v#packxcd}) ;;
              long) ;;   # --steps 1000 (below)
              tkxcd*) envs+=(STENCIL_TK_XCD=${v#tkxcd}) ;; noplace) envs+=(STENCIL_SLAB_PLACEMENTS=1) ;; place*) envs+=(STENCIL_SLAB_PLACEMENTS=${v#place}) ;; pverb) envs+=(STENCIL_SLAB_PLACE_VERBOSE=1) ;;
              sig*) envs+=(STENCIL_TK_SIG_CHUNKS=${v#sig}) ;; bsig*) envs+=(STENCIL_BOXK_SIG_CHUNKS=${v#bsig}) ;;
              xcu*x) cc=${v#xcu}; envs+=(STENCIL_SLAB_XCU=${cc%x} STENCIL_SLAB_XCU_EXCL=1) ;;
              xcu*) envs+=(STENCIL_SLAB_XCU=${v#xcu}) ;;
              *) echo "bad variant $v"; exit 2 ;;
            esac
          done
          case "$c" in C5) a="--steps 16 --warmup 4";; *) a="--steps 40 --warmup 4";; esac
          [[ "$var" == *long* ]] && a="--steps 1000 --warmup 20"
          [ "$nr" != 0 ] && a="$a --rank-of $nr"
          a="$a --allow-debug-library"
          name="xr_${c}_${nr}_${ex}_${var}${tr:+_$tr}"
          k2=1; while [ -e "$O/$name.json" ]; do k2=$((k2 + 1)); name="xr_${c}_${nr}_${ex}_${var}${tr:+_$tr}_$k2"; done
          if [ "$tr" = trace ]; then
            (cd /tmp && env "${envs[@]}" TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
               -d "$O/$name" -o run -- python3 "$R/bench.py" --config "$c" --exchange "$ex" $a --no-cpu-baseline \
               > "$O/$name.json" 2>> "$O/bench.err")
          else
            env "${envs[@]}" timeout -k 10 400 python3 bench.py --config "$c" --exchange "$ex" $a --no-cpu-baseline \
              > "$O/$name.json" 2>> "$O/bench.err"
          fi ;;
    xcdab:*) # xcdab:<dtype>:nx:ny:nz:steps -- the strip kernel's XCD-patch tile order (STENCIL_TK_XCD=w), interleaved
          IFS=':' read -r dt nx ny nz st <<< "${step#xcdab:}"
          timeout -k 10 400 python3 tools/ab.py --dtype "$dt" --grid "$nx" "$ny" "$nz" --steps "$st" --reps 5 --launches 3 \
            --variant STENCIL_TK_XCD=0 --variant STENCIL_TK_XCD=4 --variant STENCIL_TK_XCD=8 \
            --variant STENCIL_TK_XCD=16 --variant STENCIL_TK_XCD=32 > "$O/xcd_ab_${dt}_${nx}x${ny}x${nz}.txt" 2>&1 ;;
    cfgab:*) # cfgab:<dtype>:nx:ny:nz:steps:cfg1,cfg2,.. -- strip shapes (STENCIL_TK_STRIP=cfg; 1 = default), interleaved
          IFS=':' read -r dt nx ny nz st cfgs <<< "${step#cfgab:}"
          vs=(); for c in ${cfgs//,/ }; do vs+=(--variant "STENCIL_TK_STRIP=$c"); done
          timeout -k 10 400 python3 tools/ab.py --dtype "$dt" --grid "$nx" "$ny" "$nz" --steps "$st" --reps 5 --launches 3 \
            "${vs[@]}" > "$O/cfg_ab_${dt}_${nx}x${ny}x${nz}.txt" 2>&1 ;;
    kab:*) # kab:<dtype>:nx:ny:nz -- fp32 K = 5 (default) against K = 4 shapes, interleaved (debug library)
          IFS=':' read -r dt nx ny nz <<< "${step#kab:}"
          timeout -k 10 400 python3 tools/ab.py --dtype "$dt" --grid "$nx" "$ny" "$nz" --steps 5 --reps 5 --launches 3 \
            --variant STENCIL_TK_STRIP=1 --variant STEPS=4,STENCIL_TK_STRIP=1,NOCHECK=1 --variant STEPS=4,STENCIL_TK_STRIP=20808,NOCHECK=1 \
            --variant STEPS=4,STENCIL_TK_STRIP=20808,STENCIL_TK_XCD=0,NOCHECK=1 > "$O/k_ab_${dt}_${nx}x${ny}x${nz}.txt" 2>&1 ;;
    envbench:*) # envbench:<NAME=V[,NAME=V]>:<cfg> -- bench.py --config cfg with those variables (debug library allowed)
          IFS=':' read -r ev c <<< "${step#envbench:}"
          case "$c" in C1) a="--steps 100 --warmup 10";; C5) a="--steps 32 --warmup 4";; *) a="--steps 40 --warmup 4";; esac
          f="$O/envbench_${c}_${ev//[=,]/_}.json"; k2=1
          while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/envbench_${c}_${ev//[=,]/_}_$k2.json"; done
          env ${ev//,/ } timeout -k 10 400 python3 bench.py --config "$c" $a --no-cpu-baseline --allow-debug-library \
            > "$f" 2>> "$O/bench.err" ;;
    xcdpmc:*) # xcdpmc:<dtype>:nx:ny:nz:steps:w -- FETCH_SIZE / WRITE_SIZE passes of that variant's launches
          IFS=':' read -r dt nx ny nz st w <<< "${step#xcdpmc:}"
          for ctr in FETCH_SIZE WRITE_SIZE; do
            (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv \
               -d "$O/xcdpmc_${dt}_w${w}_$ctr" -o run -- python3 "$R/tools/ab.py" --dtype "$dt" --grid "$nx" "$ny" "$nz" \
               --steps "$st" --reps 1 --launches 3 --variant STENCIL_TK_XCD=$w > "$O/xcdpmc_${dt}_w${w}_$ctr.log" 2>&1) || exit 1
          done ;;
    cumask) /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o /tmp/cumask_probe &&
            timeout -k 10 60 /tmp/cumask_probe > "$O/cumask_probe.txt" 2>&1 ;;
    sustained) # the C2 job's sustained-load slowdown: telemetry (amdsmi, in-process) + a kernel trace, then a
          # GRBM_GUI_ACTIVE pass (cycles per launch), then the probe with no profiler at all
          (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/sust_trace" \
             -o run -- python3 "$R/tools/sustained_probe.py" --out "$O/sustained_trace.json" > "$O/sustained_trace.log" 2>&1) &&
          (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv \
             -d "$O/sust_pmc" -o run -- python3 "$R/tools/sustained_probe.py" --out "$O/sustained_pmc.json" \
             > "$O/sustained_pmc.log" 2>&1) &&
          timeout -k 10 200 python3 tools/sustained_probe.py --out "$O/sustained_plain.json" > "$O/sustained_plain.log" 2>&1 ;;
    envdriver:*) ev=${step#envdriver:}   # the driver's command (20 steps) with those variables (debug library)
          f="$O/envdriver_${ev//[=,]/_}.json"; k2=1
          while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/envdriver_${ev//[=,]/_}_$k2.json"; done
          env ${ev//,/ } timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
            --allow-debug-library > "$f" 2>> "$O/bench.err" ;;
    sustainedenv:*) ev=${step#sustainedenv:}   # the probe without a profiler, with those variables (debug library)
          env ${ev//,/ } timeout -k 10 200 python3 tools/sustained_probe.py --out "$O/sustained_plain_${ev//[=,]/_}.json" \
            > "$O/sustained_plain_${ev//[=,]/_}.log" 2>&1 ;;
    placeab) # bench.py --steps 1000 with 1 and 16 grid placements, alternating, three runs each
          for rep in 1 2 3; do
            for p in 1 16; do
              timeout -k 10 200 python3 bench.py --steps 1000 --warmup 20 --placements $p --no-cpu-baseline \
                > "$O/bench_1000_place${p}_$rep.json" 2>> "$O/bench.err" || exit 1
            done
          done ;;
    sqlib:*) # sqlib:<dtype>:nx:ny:nz:sweeps -- SQ / LDS / TCC counter passes of AUTO's launches of one shape
          IFS=':' read -r dt nx ny nz sw <<< "${step#sqlib:}"
          PROG=tools/time_lib.py bash profiles/collect_sq.sh "${TAG}_${dt}_${nx}x${ny}x${nz}" \
            "$R/stencil_amd/libstencil_hip.so" star "$dt" "$nx" "$ny" "$nz" "$sw" 1 > "$O/sq_${dt}_${nx}x${ny}x${nz}.log" 2>&1 ;;
    abenv:*) # abenv:<dtype>:nx:ny:nz:steps:<V1>;<V2>;.. -- tools/ab.py over variants (each NAME=V[,NAME=V]), interleaved
          IFS=':' read -r dt nx ny nz st vars <<< "${step#abenv:}"
          vs=(); IFS=';' read -r -a vl <<< "$vars"; for v in "${vl[@]}"; do vs+=(--variant "$v"); done
          f="$O/ab_${dt}_${nx}x${ny}x${nz}.txt"; k2=1; while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/ab_${dt}_${nx}x${ny}x${nz}_$k2.txt"; done
          timeout -k 10 400 python3 tools/ab.py --dtype "$dt" --grid "$nx" "$ny" "$nz" --steps "$st" --reps 7 --launches 10 \
            "${vs[@]}" > "$f" 2>&1 ;;
    pmcenv:*) # pmcenv:<dtype>:nx:ny:nz:steps:<NAME=V[,NAME=V]> -- FETCH_SIZE / WRITE_SIZE passes of tools/ab.py's launches
          IFS=':' read -r dt nx ny nz st ev <<< "${step#pmcenv:}"
          tg="${dt}_${nx}x${ny}x${nz}_${ev//[=,]/_}"
          for ctr in FETCH_SIZE WRITE_SIZE; do
            (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
               -d "$O/pmc_${tg}_$ctr" -o run -- python3 "$R/tools/ab.py" --dtype "$dt" --grid "$nx" "$ny" "$nz" \
               --steps "$st" --reps 1 --launches 5 --variant "$ev" > "$O/pmc_${tg}_$ctr.log" 2>&1) || exit 1
          done ;;
    envbench1000:*) # envbench1000:<NAME=V[,NAME=V]> -- the 1000-step C2 bench with those variables (debug library)
          ev=${step#envbench1000:}
          f="$O/envbench1000_${ev//[=,]/_}.json"; k2=1
          while [ -e "$f" ]; do k2=$((k2 + 1)); f="$O/envbench1000_${ev//[=,]/_}_$k2.json"; done
          env ${ev//,/ } timeout -k 10 300 python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline --allow-debug-library \
            > "$f" 2>> "$O/bench.err" ;;
    tierbench) STENCIL_TK_TIER=1 timeout -k 10 200 python3 bench.py --allow-debug-library --steps 1000 --warmup 20 \
             --no-cpu-baseline > "$O/bench_tier.json" 2>> "$O/bench.err" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then echo "[lease] $TAG: step $step failed rc=$rc"; exit $rc; fi
done
echo "[lease] $TAG: done $(date +%T)"
