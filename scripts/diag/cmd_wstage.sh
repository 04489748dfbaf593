set -o pipefail
bash scripts/diag/cmd_ab_libs.sh w0 w1 ab_wstage_p8.json --paths 8 --kernel ring_fwd --reps 20 || exit 1
bash scripts/diag/cmd_ab_libs.sh w0 w1 ab_wstage_p64.json --paths 64 --kernel ring_fwd --reps 20 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_x3_engine.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wstage_tests.log 2>&1 || { tail -20 gpurun_out/wstage_tests.log; exit 1; }
tail -1 gpurun_out/wstage_tests.log
