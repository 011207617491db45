set -u
mkdir -p gpurun_out
for cfg in "" "EPP_V5_BLOCK=512 EPP_WG_PER_CU5=2 EPP_V5_LDS_MIN=57344" "EPP_V5_BLOCK=512 EPP_WG_PER_CU5=2" "EPP_V5_BLOCK=512 EPP_WG_PER_CU5=2 EPP_V5_LDS_MIN=57344" "" "EPP_V5_BLOCK=512 EPP_WG_PER_CU5=2 EPP_V5_LDS_MIN=57344" "EPP_V5_BLOCK=512 EPP_WG_PER_CU5=2"; do
  env $cfg timeout -k 10 120 python bench.py --no-cpu --no-plan --no-side --steps 100 > gpurun_out/sw.json 2>/dev/null || { echo "fail $cfg"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$cfg', round(d['roofline']['kernel_ms']*1e3,3), round(d['roofline']['frac'],4))"
done
