"""Deployment and observability artefacts (reference analogue:
tests/infrastructure/test_compose.py — compose validity, ports, health
checks, dependency order, Prometheus scrape config, Grafana provisioning;
.github/workflows/ci.yml config checks).  Static checks only: Docker is not
assumed on the GPU box, so nothing here starts containers."""
from __future__ import annotations

import json
from pathlib import Path

import pytest
import yaml

from inference_arena_amd.config import get_gpu_config
from inference_arena_amd.utils.settings import Settings, _read_dotenv

ROOT = Path(__file__).resolve().parents[1]
COMPOSE = ROOT / "deploy" / "docker-compose.yml"
PROM = ROOT / "monitoring" / "prometheus.yml"
DASH = ROOT / "monitoring" / "grafana" / "dashboards"


@pytest.fixture(scope="module")
def compose():
    return yaml.safe_load(COMPOSE.read_text())


def test_compose_services_and_profiles(compose):
    svcs = compose["services"]
    assert {"init-models", "monolithic", "classification", "detection", "model-server", "gateway", "prometheus",
            "grafana"} <= set(svcs)
    prof = {n: set(s.get("profiles", [])) for n, s in svcs.items()}
    assert prof["monolithic"] == {"monolithic"}
    assert prof["detection"] == prof["classification"] == {"microservices"}
    assert prof["model-server"] == prof["gateway"] == {"triton"}
    assert prof["prometheus"] == prof["grafana"] == {"monitoring"}


def _host_ports(svc) -> set[int]:
    return {int(str(p).split(":")[0]) for p in svc.get("ports", [])}


def test_compose_ports_match_experiment_spec(compose):
    ports = get_gpu_config()["ports"]
    s = compose["services"]
    assert ports["monolithic"] in _host_ports(s["monolithic"])
    assert ports["detection"] in _host_ports(s["detection"])
    assert ports["gateway"] in _host_ports(s["gateway"])
    assert {ports["model_http"], ports["model_grpc"], ports["metrics"]} <= _host_ports(s["model-server"])
    assert s["classification"]["environment"]["PORT"] == str(ports["classification"])


def test_compose_gpu_access_and_rccl_env(compose):
    for name in ("monolithic", "classification", "detection", "model-server", "gateway", "init-models"):
        svc = compose["services"][name]
        assert "/dev/kfd" in svc["devices"] and "/dev/dri" in svc["devices"], name
        env = svc["environment"]
        if name in ("monolithic", "init-models", "model-server"):
            assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0", name


def test_compose_startup_order_and_health(compose):
    s = compose["services"]
    assert s["init-models"]["restart"] == "no"
    for name in ("monolithic", "classification", "model-server"):
        dep = s[name]["depends_on"]
        assert dep["init-models"]["condition"] == "service_completed_successfully", name
    assert s["gateway"]["depends_on"]["model-server"]["condition"] == "service_healthy"
    assert "classification" in s["detection"]["depends_on"]
    for name, path in (("monolithic", "/health"), ("model-server", "/v2/health/ready")):
        test = " ".join(s[name]["healthcheck"]["test"])
        assert path in test, name


def test_compose_commands_resolve_to_modules(compose):
    import importlib.util

    for name, svc in compose["services"].items():
        cmd = svc.get("command")
        if not cmd or cmd[0] != "python":
            continue
        if cmd[1] == "-m":
            assert importlib.util.find_spec(cmd[2]) is not None, (name, cmd[2])
        else:
            assert (ROOT / cmd[1]).exists(), (name, cmd[1])


def test_compose_network_name(compose):
    assert compose["networks"]["backend"]["name"] == "inference-arena-backend"


def test_dockerfile_builds_gfx950_extension():
    df = (ROOT / "deploy" / "Dockerfile").read_text()
    assert "PYTORCH_ROCM_ARCH=gfx950" in df and "tools/build_ext.py" in df
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in df
    for p in (8100, 8200, 8201, 8300, 8000, 8001, 8002):
        assert str(p) in df


def test_prometheus_scrape_config():
    p = yaml.safe_load(PROM.read_text())
    assert p["global"]["scrape_interval"] == "1s"
    jobs = {j["job_name"]: j for j in p["scrape_configs"]}
    assert {"prometheus", "arena-services", "arena-model-server", "arena-gpu", "cadvisor"} <= set(jobs)
    targets = [t for sc in jobs["arena-services"]["static_configs"] for t in sc["targets"]]
    assert {"monolithic:8100", "detection:8200", "gateway:8300"} <= set(targets)
    archs = {sc["labels"]["architecture"] for sc in jobs["arena-services"]["static_configs"]}
    assert archs == {"monolithic", "microservices", "triton"}
    ms = [t for sc in jobs["arena-model-server"]["static_configs"] for t in sc["targets"]]
    assert any(t.endswith(":8002") for t in ms)
    local = yaml.safe_load((ROOT / "monitoring" / "prometheus.local.yml").read_text())
    lt = [t for j in local["scrape_configs"] for sc in j["static_configs"] for t in sc["targets"]]
    assert all(t.startswith("127.0.0.1:") for t in lt)  # process mode


def _container_ports(svc) -> set[int]:
    ports = {int(str(p).split(":")[-1]) for p in svc.get("ports", [])}
    return ports | {int(p) for p in svc.get("expose", [])}


def test_every_scrape_target_resolves_to_a_compose_service(compose):
    """Inside the compose network 127.0.0.1 is the Prometheus container itself: every target must
    name a compose service that listens on that port."""
    p = yaml.safe_load(PROM.read_text())
    svcs = compose["services"]
    for job in p["scrape_configs"]:
        for sc in job["static_configs"]:
            for t in sc["targets"]:
                host, port = t.rsplit(":", 1)
                assert host in svcs, (job["job_name"], t)
                assert int(port) in _container_ports(svcs[host]), (job["job_name"], t)


def test_resource_limits_on_every_service_container(compose):
    """Reference: every container is limited to ${CONTAINER_VCPU:-2} CPUs / ${CONTAINER_MEMORY:-4096}M
    (reference architectures/monolithic/docker-compose.yml:95-98)."""
    for name in ("init-models", "monolithic", "classification", "detection", "model-server", "gateway",
                 "gpu-exporter"):
        lim = compose["services"][name]["deploy"]["resources"]["limits"]
        assert lim["cpus"].startswith("${CONTAINER_VCPU") and lim["memory"].startswith("${CONTAINER_MEMORY"), name
    env = (ROOT / ".env.example").read_text()
    assert "CONTAINER_VCPU=" in env and "CONTAINER_MEMORY=" in env


def test_monitoring_stack_has_cadvisor_and_gpu_exporter(compose):
    s = compose["services"]
    assert s["cadvisor"]["privileged"] is True and "8080:8080" in s["cadvisor"]["ports"]
    assert s["gpu-exporter"]["command"][:3] == ["python", "-m", "inference_arena_amd.metrics.gpu"]
    assert "/dev/kfd" in s["gpu-exporter"]["devices"]


def test_per_arm_compose_files_in_sync():
    import subprocess
    import sys

    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "gen_compose.py"), "--check"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    for arm, must in (("monolithic", {"init-models", "monolithic"}), ("microservices", {"classification", "detection"}),
                      ("triton", {"model-server", "gateway"}), ("infra", {"prometheus", "grafana", "cadvisor"})):
        doc = yaml.safe_load((ROOT / "deploy" / "compose" / f"{arm}.yml").read_text())
        assert must <= set(doc["services"]), arm
        assert doc["networks"]["backend"]["name"] == "inference-arena-backend"


@pytest.mark.parametrize("arch", ["monolithic", "microservices", "triton"])
def test_grafana_dashboards(arch):
    d = json.loads((DASH / f"{arch}.json").read_text())
    # the reference's dashboard uids (infrastructure/grafana/provisioning/dashboards/infrastructure-*.json)
    assert d["uid"] == {"monolithic": "inference-arena-mono", "microservices": "inference-arena-micro",
                        "triton": "inference-arena-triton"}[arch]
    titles = [p["title"] for p in d["panels"]]
    for t in ("Throughput (req/s)", "End-to-end latency (ms)", "GPU utilization (%)", "Container CPU (%)",
              "Container memory (MB)"):
        assert t in titles, (arch, t)
    for p in d["panels"]:
        for tgt in p.get("targets", []):
            expr = tgt.get("expr", "")
            assert expr, (arch, p["title"])
            assert "container_id=\"" not in expr, "dashboards select by label, not hard-coded container ids"


def test_grafana_provisioning():
    prov = ROOT / "monitoring" / "grafana" / "provisioning"
    ds = yaml.safe_load((prov / "datasources" / "prometheus.yml").read_text())["datasources"][0]
    assert ds["type"] == "prometheus" and ds["jsonData"]["timeInterval"] == "1s"
    db = yaml.safe_load((prov / "dashboards" / "arena.yml").read_text())["providers"][0]
    assert db["type"] == "file"


def test_ci_workflow_runs_cpu_and_gpu_tiers():
    w = yaml.safe_load((ROOT / ".github" / "workflows" / "ci.yml").read_text())
    assert {"cpu-tests", "gpu-tests", "code-quality", "build", "validate-config", "program-bounds", "compose-check",
            "security", "single-source-of-truth", "summary"} <= set(w["jobs"])
    v = yaml.safe_load((ROOT / ".github" / "workflows" / "validate-experiment-config.yml").read_text())
    assert "validate" in v["jobs"]
    text = (ROOT / ".github" / "workflows" / "ci.yml").read_text()
    assert 'not gpu' in text and "-m gpu" in text


def test_env_template_keys_are_known_settings():
    env = _read_dotenv(ROOT / ".env.example")
    known = set(Settings.model_fields) | {"ARENA_FUSE_IR", "ARENA_CONV_IMPL", "HSA_ENABLE_IPC_MODE_LEGACY",
                                          "MASTER_ADDR", "GRAFANA_ADMIN_USER", "GRAFANA_ADMIN_PASSWORD",
                                          "PROMETHEUS_PORT", "GRAFANA_PORT", "MINIO_INTERNAL_ENDPOINT",
                                          "MINIO_ACCESS_KEY", "MINIO_SECRET_KEY", "MINIO_BUCKET", "MINIO_SECURE",
                                          # compose interpolation (deploy/docker-compose.yml)
                                          "CONTAINER_VCPU", "CONTAINER_MEMORY", "GPUS", "LAST_GPU", "ARENA_DTYPE",
                                          "ARENA_DECODE_PROCS"}
    assert set(env) <= known, set(env) - known
    # the template's values are valid settings (inline comments stripped)
    s = Settings(**{k: v for k, v in env.items() if k in Settings.model_fields})
    assert s.MODELS_DIR == "model_repository"
    assert s.ARENA_MAX_BATCH == 32 and s.ARENA_CROP_TRANSPORT == "jpeg"


def test_dotenv_parsing(tmp_path):
    p = tmp_path / ".env"
    p.write_text('# comment\nA=1   # trailing\nB="x # not a comment"\nC=\'q\'\n\nD=plain\nE=a=b\nbad line\n')
    env = _read_dotenv(p)
    assert env == {"A": "1", "B": "x # not a comment", "C": "q", "D": "plain", "E": "a=b"}


def test_settings_env_precedence(tmp_path, monkeypatch):
    p = tmp_path / ".env"
    p.write_text("PORT=9100\nLOG_LEVEL=DEBUG\n")
    monkeypatch.setenv("PORT", "9200")
    s = Settings.from_env(p)
    assert s.PORT == 9200 and s.LOG_LEVEL == "DEBUG"
    s2 = Settings.from_env(p, PORT=9300)
    assert s2.PORT == 9300
