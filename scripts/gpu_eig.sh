#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 120 ./tools/eig_probe 925 8 > gpurun_out/eig925.log 2>&1 && cat gpurun_out/eig925.log &&
timeout -k 10 120 ./tools/eig_probe 256 32 > gpurun_out/eig256.log 2>&1 && cat gpurun_out/eig256.log
