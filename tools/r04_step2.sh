# round 4, step 2: the HBM stream-mix ceilings (incl. the Poisson catch-up
# kernels' 4R+2W and 5R+2W), then one rank's iteration at G = 1/2/4/8 without
# the collectives, timed and kernel-traced (the scale model's inputs)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 120 tools/microbench/_bin/hbm_mix_peak > gpurun_out/r04_hbm_mix.json || exit 1
cat gpurun_out/r04_hbm_mix.json
rm -f gpurun_out/r04_rank_iteration.jsonl
for g in 2 4 8; do
  timeout -k 10 120 tools/microbench/_bin/rank_iteration $g 60 >> gpurun_out/r04_rank_iteration.jsonl || exit 1
done
for g in 2 4 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r04_rank_kt$g -o kt --output-format csv -- \
      tools/microbench/_bin/rank_iteration $g 60 > /dev/null || exit 1
done
cat gpurun_out/r04_rank_iteration.jsonl
