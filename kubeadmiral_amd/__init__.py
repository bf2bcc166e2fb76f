"""kubeadmiral_amd — MI355X-native batch scheduler for KubeAdmiral's scheduling framework."""
