set -e
mkdir -p gpurun_out
(timeout -k 10 100 tools_dev/garbage/garbage mfma 40 > gpurun_out/r02i_g.log 2>&1 &)
sleep 3
for v in nopk v0; do
  for op in ff1x oproj; do
    echo "$v $(timeout -k 10 30 tools_dev/garbage/victim3_$v 6 $op)" >> gpurun_out/r02i.log
  done
done
sleep 1
