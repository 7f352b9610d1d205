set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 > gpurun_out/fin_bench.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/fin_bench.json'));print('bench', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fin -o run --output-format csv -- python3 bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 20 > /dev/null 2>&1
