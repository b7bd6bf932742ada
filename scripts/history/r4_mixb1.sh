#!/bin/bash
# Mixtral-8x7B batch-1 decode window on the current tree
bash scripts/window.sh mixb1 40 --model mixtral-8x7b --batch 1
