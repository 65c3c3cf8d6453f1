#!/bin/bash
# Round-6 closing measurement set on this tree's build (scripts/gpu_final.sh with the r06y workloads).
OUT=${OUT:-gpurun_out/r06z} PROF_SET="default:;drv:--steps 20 --warmup 5;c1:--basin bs;c2:--n 1024;c3:--n 2048 --blocks 2x2;c4:--blocks 4x2;c4topo:--blocks 4x2 --topography;c5:--basin bs_tr --blocks 4x2;general:--no-known-constants;lone:--box 1024x2048;topo:--topography" bash scripts/gpu_final.sh
