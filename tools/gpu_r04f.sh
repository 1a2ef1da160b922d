#!/bin/bash
# round-4 iteration batch: latency kernel v2 (parity + timing + throughput A/B), PPO KC A/B, HF pass-2 A/B
set -o pipefail
bash tools/gpu_lat_ab.sh && bash tools/gpu_ppo_ab.sh && A=p2 CFGS="C4 C5" STEPS=200 bash tools/gpu_ab_quick.sh
