"""kubelet device-plugin control plane."""
