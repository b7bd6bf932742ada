# Operator image (mlopamd/mlflow-operator): the control plane only (no GPU, no torch).
# manifests/operator-deployment.yaml runs it as
#   python -m mlopamd.controller run --all-namespaces
#   docker build -f docker/operator.Dockerfile -t mlopamd/mlflow-operator:0.1.0 .
FROM python:3.10-slim
ENV PYTHONUNBUFFERED=1
WORKDIR /opt/mlopamd
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/__init__.py research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/controller/ research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/controller/
# the placement planner reads the model shapes; models/__init__.py and config.py import without torch
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/models/__init__.py research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/models/config.py research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/models/
COPY manifests/ manifests/
# OPERATOR_PIP (tests/test_packaging_cpu.py imports the operator with only these + the stdlib)
RUN ln -s research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd mlopamd \
 && pip install --no-cache-dir pyyaml numpy aiohttp prometheus_client
ENV PYTHONPATH=/opt/mlopamd
USER 65532:65532
EXPOSE 8080
ENTRYPOINT ["python", "-m", "mlopamd.controller"]
CMD ["run", "--all-namespaces"]
