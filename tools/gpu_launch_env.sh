set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/lp.txt
for e in "X=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0"; do
  echo "== $e" >> $O
  env $e timeout -k 10 60 tools/launch_probe >> $O 2>&1 || exit 1
done
for e in "X=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  echo "== chain $e" >> $O
  env $e timeout -k 10 120 python -u tools/chain_probe.py 50 add,mm768,ln_mm768,mlp >> $O 2>&1 || exit 1
done
