# step time with the weight-gradient GEMMs forced onto one tile variant (CAPGEN_DW_VARIANT)
for v in 0 1 3 10 9 2 6 203 210; do echo -n "dw variant $v: "; CAPGEN_DW_VARIANT=$v timeout -k 10 100 python bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])" || exit 1; done
