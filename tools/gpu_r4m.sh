#!/bin/bash
# second residual deposit (decoder skip) + GN tests, then the profiler stacks
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "residual_grad_slot or group_norm or cat_gn or full_model or model_hip_vs or graph_train_step" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
