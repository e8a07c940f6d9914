for c in cfg3_resnet50_r4 cfg2_resnet50_r1 cfg4_llama_r2_bf16; do
  for v in "PSGD_W1_OVERLAP=1 PSGD_BUCKETS=2" "PSGD_W1_OVERLAP=1 PSGD_BUCKETS=3" "PSGD_W1_OVERLAP=1 PSGD_BUCKETS=4" "PSGD_W1_OVERLAP=0"; do
    env $v timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
    echo "$c [$v] $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/b.log') if l.startswith('{')][0]);print('cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],d['config']['w1_bucket_overlap'],d['config']['buckets'])")"
  done
done
