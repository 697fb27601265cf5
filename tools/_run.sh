timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; exit $rc
