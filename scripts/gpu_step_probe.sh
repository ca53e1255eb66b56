# host wall time per phase of a bench step, with and without torch initialised; bench per-step times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/step_probe.py --size-gb 10 --torch > gpurun_out/step_probe_torch.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_steps.log 2>&1 || exit 2
