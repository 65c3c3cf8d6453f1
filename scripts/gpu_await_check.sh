set -e
mkdir -p gpurun_out/await
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair.py -k "first_call or pair_steps_match or default_threshold or counts_blowup or one_step_calls" > gpurun_out/await/pytest.txt 2>&1
OUT=gpurun_out/await bash scripts/gpu_clock_probe.sh
for r in 1 2; do
timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/await/drv_$r.json 2> gpurun_out/await/drv_$r.err
timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/await/def_$r.json 2> gpurun_out/await/def_$r.err
done
tail -2 gpurun_out/await/pytest.txt
for f in gpurun_out/await/*_?.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],5), d.get('stage_ms'))" $f; done
