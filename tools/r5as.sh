set -o pipefail
mkdir -p gpurun_out/r5au
for v in off fc2,proj fc2,fc1,proj fc2,proj,qkv; do
  MIA_MX_DGRAD=$( [ $v = off ] && echo "" || echo $v ) timeout -k 10 400 python -u bench.py --model ast-fp8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5au/b_$v.json 2> gpurun_out/r5au/b_$v.err || exit 1
done
