#!/bin/bash
# tests/golden/c1_loopback.npz: 10,000 64-B TCP frames injected on lo and captured back
# (examples/capture_sessions.py; needs CAP_NET_RAW, no GPU).  BASELINE.json configs[0].
set -e
cd "$(dirname "$0")/.."
python examples/capture_sessions.py --packets 10000 --flows 100 --capture-only --save tests/golden/c1_loopback.npz
