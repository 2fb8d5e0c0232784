set -u
mkdir -p gpurun_out
B="--no-cpu-baseline --no-host --no-other-mode --no-single-launch"
for a in "--config 2 --rotate 8 --steps 240 --no-imix" "--config 2 --rotate 12 --steps 240 --no-imix" "--config 2 --rotate 8 --steps 240 --no-imix" "--config 2 --rotate 12 --steps 240 --no-imix" "--config 3 --rotate 4 --steps 240" "--config 3 --rotate 8 --steps 240" "--config 3 --rotate 12 --steps 240"; do
  timeout -k 10 200 python bench.py $a $B > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo FAIL $a; cat gpurun_out/sw.err | tail; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$a',d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_per_launch'])"
done
