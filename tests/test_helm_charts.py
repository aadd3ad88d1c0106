"""The bundled Helm charts (KubeApps-Plus store content) rendered by a Go-template interpreter
(tests/helm_template.py) with default and multi-node values, parsed as YAML and checked: torchrun arguments that
the training CLI actually accepts, one pod per node with ``amd.com/gpu`` limits and a memory-backed /dev/shm,
the rendezvous Service + Indexed Job for multi-node jobs, checkpoint PVC wiring, and the serving Deployment's
GPU request / readiness probe / arguments."""
import os

import pytest

from helm_template import TemplateError, render_chart, render_docs

CHARTS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "kubeoperator_amd/control/resources/kubeasz/roles/kubeapps/files/charts")


def _kind(docs, kind):
    out = [d for d in docs if d["kind"] == kind]
    assert len(out) == 1, [d["kind"] for d in docs]
    return out[0]


def _trainer_args(job):
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["python", "-m", "torch.distributed.run"]
    args = c["args"]
    i = args.index("-m")
    assert args[i + 1] == "kubeoperator_amd.train.cli"
    return args[:i], args[i + 2:], c


def test_training_chart_single_node():
    docs = render_docs(os.path.join(CHARTS, "pytorch-rocm-train"))
    assert [d["kind"] for d in docs] == ["Job"]  # no rendezvous Service for one node
    job = docs[0]
    launcher, train, c = _trainer_args(job)
    assert "--standalone" in launcher and "--nproc-per-node=8" in launcher and "--nnodes=1" in launcher
    from kubeoperator_amd.train.cli import build_parser

    a = build_parser().parse_args(train)  # every rendered flag exists in the CLI (argparse exits otherwise)
    assert a.model == "llama3_8b" and a.seq == 8192 and a.accum == 4 and a.dp == "auto" and a.tp == 1
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["TORCH_NCCL_HIGH_PRIORITY"] == "1"
    spec = job["spec"]["template"]["spec"]
    shm = next(v for v in spec["volumes"] if v["name"] == "dshm")
    assert shm["emptyDir"] == {"medium": "Memory", "sizeLimit": "64Gi"}
    assert {"name": "dshm", "mountPath": "/dev/shm"} in c["volumeMounts"]
    assert spec["nodeSelector"] == {"kubeoperator.io/gpu": "true"} and spec["hostIPC"] is True
    assert job["spec"]["completions"] == 1 and "completionMode" not in job["spec"]
    ann = job["spec"]["template"]["metadata"]["annotations"]
    assert ann == {"prometheus.io/scrape": "true", "prometheus.io/port": "9400"}


def test_training_chart_multi_node_rendezvous_and_checkpoint():
    docs = render_docs(os.path.join(CHARTS, "pytorch-rocm-train"),
                       {"nodes": 4, "checkpoint": {"enabled": True}, "tensorParallel": 2, "recompute": True},
                       release="llama")
    svc, job = _kind(docs, "Service"), _kind(docs, "Job")
    name = job["metadata"]["name"]
    assert svc["metadata"]["name"] == name and svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["selector"] == {"job-name": name}
    assert job["spec"]["completionMode"] == "Indexed" and job["spec"]["completions"] == 4
    assert job["spec"]["parallelism"] == 4
    spec = job["spec"]["template"]["spec"]
    assert spec["subdomain"] == name and job["spec"]["template"]["metadata"]["labels"] == {"job-name": name}
    launcher, train, c = _trainer_args(job)
    assert "--standalone" not in launcher
    assert f"--rdzv-endpoint={name}-0.{name}:29500" in launcher  # pod 0's DNS name under the headless service
    assert "--rdzv-backend=c10d" in launcher and "--node-rank=$(JOB_COMPLETION_INDEX)" in launcher
    from kubeoperator_amd.train.cli import build_parser

    a = build_parser().parse_args(train)
    assert a.resume and a.ckpt_dir == "/ckpt" and a.ckpt_every == 500 and a.tp == 2 and a.recompute == 1
    ck = next(v for v in spec["volumes"] if v["name"] == "ckpt")
    assert ck["persistentVolumeClaim"]["claimName"] == f"{name}-ckpt"
    assert {"name": "ckpt", "mountPath": "/ckpt"} in c["volumeMounts"]


def test_training_chart_name_is_truncated_to_a_dns_label():
    docs = render_docs(os.path.join(CHARTS, "pytorch-rocm-train"), release="r" * 80)
    n = docs[0]["metadata"]["name"]
    assert len(n) <= 63 and not n.endswith("-")


def test_serving_chart():
    docs = render_docs(os.path.join(CHARTS, "pytorch-rocm-serve"), {"checkpoint": {"dir": "/ckpt", "pvc": "llama-ckpt"},
                                                                    "hipGraph": True, "replicas": 2})
    dep, svc = _kind(docs, "Deployment"), _kind(docs, "Service")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 1 and dep["spec"]["replicas"] == 2
    assert c["readinessProbe"]["httpGet"]["path"] == "/healthz"
    from kubeoperator_amd.serve.server import build_parser

    a = build_parser().parse_args(c["args"])
    assert a.ckpt == "/ckpt" and a.graph == 1 and a.port == 8000 and a.max_batch == 64
    assert dep["spec"]["template"]["spec"]["volumes"][0]["persistentVolumeClaim"]["claimName"] == "llama-ckpt"
    assert svc["spec"]["ports"][0]["port"] == 8000
    plain = render_docs(os.path.join(CHARTS, "pytorch-rocm-serve"))
    pc = _kind(plain, "Deployment")["spec"]["template"]["spec"]
    assert "volumes" not in pc and "--ckpt" not in " ".join(pc["containers"][0]["args"])


def test_nginx_chart():
    docs = render_docs(os.path.join(CHARTS, "nginx"))
    dep, svc = _kind(docs, "Deployment"), _kind(docs, "Service")
    assert dep["spec"]["template"]["spec"]["containers"][0]["image"] == "nginx:1.27-alpine"
    assert svc["spec"]["type"] == "ClusterIP"


def test_renderer_rejects_what_it_does_not_implement(tmp_path):
    (tmp_path / "templates").mkdir()
    (tmp_path / "Chart.yaml").write_text("name: x\nversion: 0.1.0\n")
    (tmp_path / "values.yaml").write_text("a: 1\n")
    (tmp_path / "templates" / "t.yaml").write_text("x: {{ include \"foo\" . }}\n")
    with pytest.raises(TemplateError):
        render_chart(str(tmp_path))
