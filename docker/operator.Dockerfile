# Operator image (mlopamd/mlflow-operator): the control plane only (no GPU, no torch).
# manifests/operator-deployment.yaml runs it as
#   python -m mlopamd.controller run --all-namespaces
#   docker build -f docker/operator.Dockerfile -t mlopamd/mlflow-operator:0.1.0 .
FROM python:3.10-slim
ENV PYTHONUNBUFFERED=1
WORKDIR /opt/mlopamd
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/__init__.py research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/
COPY research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/controller/ research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd/controller/
COPY manifests/ manifests/
RUN ln -s research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd mlopamd \
 && pip install --no-cache-dir pyyaml numpy
ENV PYTHONPATH=/opt/mlopamd
USER 65532:65532
EXPOSE 8080
ENTRYPOINT ["python", "-m", "mlopamd.controller"]
CMD ["run", "--all-namespaces"]
