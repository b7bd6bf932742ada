#!/bin/bash
# batch-64 decode window on the round-4 tree
bash scripts/window.sh b64 20 --batch 64 && bash scripts/window.sh b16 20 --batch 16
