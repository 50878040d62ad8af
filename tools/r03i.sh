set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
timeout -k 10 400 python -u -m pytest tests/test_cli.py tests/test_gpu_seqparse.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i/pytest_cli.log 2>&1 || { tail -30 gpurun_out/r03i/pytest_cli.log; exit 1; }
tail -2 gpurun_out/r03i/pytest_cli.log
timeout -k 10 200 bash tools/cli_trace.sh gpurun_out/r03i/cli || exit 1
NO_TRACE=1 CLI_ENV="FPMASH_MSH_WRITE=pwrite" timeout -k 10 200 bash tools/cli_trace.sh gpurun_out/r03i/cli_pwrite || exit 1
NO_TRACE=1 CLI_ENV="HSA_ENABLE_SDMA=0" timeout -k 10 200 bash tools/cli_trace.sh gpurun_out/r03i/cli_nosdma || exit 1
