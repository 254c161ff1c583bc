#!/bin/bash
# One-shot cluster deploy for mihvd (counterpart of the reference's deploy_stack.sh):
#   1. namespaces (ml-ops, loki, mpi-operator)       2. Loki + Promtail + Grafana (log observability,
#      deploy/loki-stack-values.yaml: rank label from the log prefix; dashboard deploy/grafana/)
#   3. Kubeflow MPI Operator (pinned, not `master`) 4. checkpoint PVC + the MPIJob
# Every setting can be overridden from the environment; DRY_RUN=1 prints the commands instead.
set -euo pipefail

NAMESPACE=${NAMESPACE:-ml-ops}
LOKI_NAMESPACE=${LOKI_NAMESPACE:-loki}
MPI_NAMESPACE=${MPI_NAMESPACE:-mpi-operator}
MPI_OPERATOR_VERSION=${MPI_OPERATOR_VERSION:-v0.6.0}
LOKI_PERSISTENCE_SIZE=${LOKI_PERSISTENCE_SIZE:-5Gi}
JOB_MANIFEST=${JOB_MANIFEST:-$(dirname "$0")/mpijob-mi355x.yaml}
PVC_MANIFEST=${PVC_MANIFEST:-$(dirname "$0")/checkpoint-pvc.yaml}
LOKI_VALUES=${LOKI_VALUES:-$(dirname "$0")/loki-stack-values.yaml}
DASHBOARD=${DASHBOARD:-$(dirname "$0")/grafana/mihvd-dashboard.json}
IMAGE=${IMAGE:-mihvd:latest}
DRY_RUN=${DRY_RUN:-0}

run() {
  if [ "$DRY_RUN" = "1" ]; then echo "+ $*"; else "$@"; fi
}

echo "Creating namespaces..."
for ns in "$NAMESPACE" "$LOKI_NAMESPACE" "$MPI_NAMESPACE"; do
  run kubectl create namespace "$ns" || true
done

echo "Installing the Loki stack (Loki + Promtail + Grafana)..."
run helm repo add grafana https://grafana.github.io/helm-charts || true
run helm repo update
run helm upgrade --install loki grafana/loki-stack \
  --namespace "$LOKI_NAMESPACE" \
  -f "$LOKI_VALUES" \
  --set grafana.enabled=true \
  --set promtail.enabled=true \
  --set loki.persistence.enabled=true \
  --set loki.persistence.size="$LOKI_PERSISTENCE_SIZE" \
  --wait

echo "Provisioning the Grafana dashboard (Loki queries over the structured training logs)..."
if [ "$DRY_RUN" = "1" ]; then
  echo "+ kubectl create configmap mihvd-dashboard -n $LOKI_NAMESPACE --from-file=$DASHBOARD --dry-run=client -o yaml | kubectl apply -f -"
  echo "+ kubectl label configmap mihvd-dashboard -n $LOKI_NAMESPACE grafana_dashboard=1 --overwrite"
else
  kubectl create configmap mihvd-dashboard -n "$LOKI_NAMESPACE" --from-file="$DASHBOARD" \
    --dry-run=client -o yaml | kubectl apply -f -
  kubectl label configmap mihvd-dashboard -n "$LOKI_NAMESPACE" grafana_dashboard=1 --overwrite
fi

echo "Installing the MPI Operator ${MPI_OPERATOR_VERSION}..."
run kubectl apply --server-side -f \
  "https://raw.githubusercontent.com/kubeflow/mpi-operator/${MPI_OPERATOR_VERSION}/deploy/v2beta1/mpi-operator.yaml"

echo "Deploying the mihvd MNIST job (image ${IMAGE})..."
run kubectl apply -n "$NAMESPACE" -f "$PVC_MANIFEST"
if [ "$DRY_RUN" = "1" ]; then
  echo "+ sed s#mihvd:latest#${IMAGE}# $JOB_MANIFEST | kubectl apply -n $NAMESPACE -f -"
else
  sed "s#mihvd:latest#${IMAGE}#g" "$JOB_MANIFEST" | kubectl apply -n "$NAMESPACE" -f -
fi

echo "Done. Logs: kubectl logs -n $NAMESPACE -l role=launcher -f  |  Grafana/Loki: {namespace=\"$NAMESPACE\"}"
