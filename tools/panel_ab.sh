# Dev A/B (round 6, verdict item 7): the dense step with the panel kernel's RHS operand
# (product) against a timing-only build without it (libgpmi_norhs.so: wrong r, so the
# bench's parity checks are not meaningful there), alternating, plus a kernel trace of
# each for the panel time per step.   bash tools/panel_ab.sh <name>
set -o pipefail
D=gpurun_out/${1:?name}
mkdir -p $D
for rep in 1 2; do
  for v in base norhs; do
    if [ $v = norhs ]; then export GPMI_LIB_VARIANT=norhs; else unset GPMI_LIB_VARIANT; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-band --no-sparse --no-extras --out-json $D/dense_${v}_$rep.json > $D/dense_${v}_$rep.err 2>&1 || { tail -5 $D/dense_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],1), d['roofline']['frac'])" $D/dense_${v}_$rep.json "$v"
  done
done
for v in base norhs; do
  if [ $v = norhs ]; then export GPMI_LIB_VARIANT=norhs; else unset GPMI_LIB_VARIANT; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-band --no-sparse --no-extras --out-json $D/dense_${v}_prof.json > $D/prof_$v.err 2>&1 || { tail -5 $D/prof_$v.err; exit 1; }
  grep -E "panel_kernel|diag_block|syrk_kernel" $D/prof_$v/run_kernel_stats.csv | cut -d, -f1-4
  find $D/prof_$v -name '*kernel_trace.csv' -delete
done
