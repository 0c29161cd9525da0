#!/bin/bash
# round 2 (u): PMC passes of the K=12 launch (the dominant depth of the driver's 20-turn run:
# 12 + 8), summarised into profiles/pmc_traffic.json key 65536x65536_k12 on the CPU side
set -e
./scripts/pmc_passes.sh 12
