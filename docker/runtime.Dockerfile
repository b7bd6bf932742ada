# Predictor image (mlopamd/runtime-rocm): the PyTorch-ROCm serving runtime with the gfx950
# HIP kernels compiled in.  Referenced by the SeldonDeployments the operator emits
# (controller/seldon.py build_predictor, env MLOP_RUNTIME_IMAGE) and started as
#   python -m mlopamd.runtime.server --port 9000 --tp <TP>
# (TP > 1: one process per GPU, RCCL over xGMI; the pod requests amd.com/gpu = TP).
#   docker build -f docker/runtime.Dockerfile -t mlopamd/runtime-rocm:0.1.0 .
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTHONUNBUFFERED=1
WORKDIR /opt/mlopamd
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/ ./research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/
COPY __graft_entry__.py bench.py ./
COPY scripts/build_sanitized.sh scripts/
COPY tests/native/ tests/native/
RUN ln -s research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd mlopamd \
 && pip install --no-cache-dir fastapi uvicorn safetensors tokenizers prometheus_client pyyaml \
 && python -c "from mlopamd.ops.build import build; print(build())"
ENV PYTHONPATH=/opt/mlopamd
EXPOSE 9000
HEALTHCHECK CMD python -c "import urllib.request as u; u.urlopen('http://127.0.0.1:9000/v2/health/live')"
ENTRYPOINT ["python", "-m", "mlopamd.runtime.server"]
CMD ["--port", "9000"]
