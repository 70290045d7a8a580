"""Deployment artefacts are consistent with the plugin's flag surface."""
import glob
import os
import re

import yaml

from amdvgpu.plugin.config import build_parser, parse_config

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _known_flags():
    flags = set()
    for a in build_parser()._actions:
        flags.update(s for s in a.option_strings if s.startswith("--"))
    return flags


def test_static_manifests_parse_and_args_are_valid():
    files = glob.glob(os.path.join(REPO, "deployments", "static", "*.yml"))
    assert len(files) >= 3
    for f in files:
        docs = [d for d in yaml.safe_load_all(open(f)) if d]
        ds = [d for d in docs if d["kind"] == "DaemonSet"]
        assert ds, f
        for c in ds[0]["spec"]["template"]["spec"]["containers"]:
            if "args" in c:
                parse_config(c["args"], environ={})


def test_helm_template_flags_exist():
    tpl = open(os.path.join(REPO, "deployments", "helm", "amd-vgpu-device-plugin", "templates",
                            "daemonset.yml")).read()
    used = set(re.findall(r'"(--[a-z-]+)=', tpl))
    assert used and used <= _known_flags(), used - _known_flags()
    values = yaml.safe_load(open(os.path.join(REPO, "deployments", "helm", "amd-vgpu-device-plugin",
                                              "values.yaml")))
    for key in re.findall(r"\.Values\.([A-Za-z]+)", tpl):
        assert key in values, key


def test_preload_file_points_at_container_shim():
    from amdvgpu.plugin.contract import CONTAINER_SHIM
    assert open(os.path.join(REPO, "vgpu", "ld.so.preload")).read().strip() == CONTAINER_SHIM


def test_image_build_inputs_exist():
    """Static check of docker/Dockerfile (no container engine in CI's first stage): every
    COPY source exists, the make targets are real targets, and the entrypoint installs
    exactly what the build produces."""
    import re
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    df = open(os.path.join(repo, "docker", "Dockerfile")).read()
    for src in re.findall(r"^COPY (?!--from)(\S+)", df, re.M):
        assert os.path.exists(os.path.join(repo, src.rstrip("/"))), src
    targets = re.findall(r"\.\./4paradigm-k8s-device-plugin_amd/lib/(\S+)", df)
    assert set(targets) == {"libvgpu_hip.so", "libvgpu_region.so", "vgpuctl", "vgpu-ledger", "vgpu-validate"}
    for t in targets:  # make knows how to build each one (dry run)
        rc = subprocess.call(["make", "-n", "-C", os.path.join(repo, "native"),
                              f"../4paradigm-k8s-device-plugin_amd/lib/{t}"], stdout=subprocess.DEVNULL)
        assert rc == 0, t
    ep = open(os.path.join(repo, "docker", "entrypoint.sh")).read()
    installed = re.search(r"for f in ([^;]+);", ep).group(1).split()
    # The ledger daemon runs inside the plugin's own container; nothing mounts it into pods.
    assert set(installed) == (set(targets) - {"vgpu-ledger"}) | {"ld.so.preload"}
    assert "lock" in ep and "containers" in ep


def test_image_rehearsal_builds_and_entrypoint_installs(tmp_path):
    """docker/Dockerfile replayed stage by stage without a container engine
    (tools/image_rehearsal.py): the build stage compiles the product from the filtered
    context, the runtime stage's entrypoint installs the data plane and starts the
    plugin's CLI (--help)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import image_rehearsal
    stages, final = image_rehearsal.rehearse(str(tmp_path), log=lambda *_: None)
    out = image_rehearsal.check_runtime(final, str(tmp_path), log=lambda *_: None)
    assert "--device-split-count" in out and "--cu-mode" in out
