# usage: bash tools/tune_mmv.sh "PD:BLOCKS ..."  -- sweeps the streaming GEMV launch parameters
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_mul_mat_gpu.py -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; tail -1 gpurun_out/gpu_tests.log
for cfg in $1; do
  pd=${cfg%%:*}; blk=${cfg##*:}
  r=$(GGML_MI355X_MMV_BLOCKS=$blk GGML_MI355X_MMV_VARIANT=$pd timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu --no-sweep 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['event_ms_per_step'])")
  echo "pd=$pd blocks=$blk -> $r"
done
