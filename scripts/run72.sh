#!/bin/bash
# HF checkpoints (transformers-saved tiny Llama / Mixtral) served by the GPU engine.
source scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pytest_loader 300 python -u -m pytest tests/test_loader_gpu.py -x -v --timeout 200 --timeout-method thread
