set -o pipefail
mkdir -p gpurun_out/r06b
Q="--extra none --single-steps 0 --icp-jobs 0 --cpu-scans 0 --modes-steps 0 --profile-steps 4 --steps 12 --warmup 3"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --extra none --icp-jobs 0 --cpu-scans 0 --single-steps 0 --detail-out gpurun_out/r06b/d512.json > gpurun_out/r06b/b512.out 2> gpurun_out/r06b/b512.err &&
for S in 256 384 640; do timeout -k 10 300 python -u bench.py $Q --streams $S --detail-out gpurun_out/r06b/d$S.json > gpurun_out/r06b/b$S.out 2> gpurun_out/r06b/b$S.err || exit $?; done
