#!/bin/bash
# r3c (changed-area tests, BERT/GPT benches, BERT profile) then r3d (GEMM A/B + counters, ResNet/GPT profiles)
bash scripts/gpu_r3c.sh r3c && bash scripts/gpu_r3d.sh r3d
