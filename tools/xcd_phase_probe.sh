set -o pipefail
mkdir -p gpurun_out/r06_xcd
P=tools/xcd_phase_probe
for a in "-W 16384 -R 16384" "-W 16384 -R 16384 --side" "-W 9216 -R 294912" "-W 9216 -R 294912 --side" "-W 36864 -R 294912 --side" "-W 1024 -R 1024" "-W 1024 -R 1024 --side"; do
  timeout -k 10 60 $P $a >> gpurun_out/r06_xcd/probe.txt 2>&1 || { echo "rc $? on $a"; exit 1; }
done
cat gpurun_out/r06_xcd/probe.txt
