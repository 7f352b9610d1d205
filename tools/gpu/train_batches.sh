set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r06tb; mkdir -p $o
B="bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 2 --warmup 1"
for rep in 1 2; do
 for cfg in "SML_LIB=abx/g16/speedy-ml-1_amd/lib/libspeedyml.so:4" "SML_LIB=abx/g16/speedy-ml-1_amd/lib/libspeedyml.so:1" "SML_AB=m4:1" "SML_LIB=abx/g16/speedy-ml-1_amd/lib/libspeedyml.so:2"; do
  e=${cfg%%:*}; nb=${cfg##*:}; f=$o/$(echo $e | tr -c 'a-z0-9' _)_${nb}_$rep
  env $e timeout -k 10 400 python -u $B --train-batches $nb > $f.json 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d['training']; print('[$cfg] rep $rep gram', t['gram_ms'], t['roofline']['frac'], 'solve', t['solve_ms'], t['solve_roofline']['frac'], t['solve_info_ok'])"
 done
done
