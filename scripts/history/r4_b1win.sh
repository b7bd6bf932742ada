#!/bin/bash
# batch-1 and batch-4 decode windows with the GEMV norm chain
bash scripts/window.sh b1chain 40 --batch 1 && bash scripts/window.sh b4chain 40 --batch 4
