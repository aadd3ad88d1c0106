"""KubeOperator-compatible control plane (cluster lifecycle manager) of kubeoperator_amd."""
