#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_graph.py -x -q -p no:cacheprovider > gpurun_out/tests_graph.log 2>&1
echo "graph rc=$?"
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider --deselect tests/test_gpu_graph.py > gpurun_out/tests_gpu.log 2>&1
echo "pytest rc=$?"
