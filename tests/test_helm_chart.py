"""The Helm chart, rendered (ncc/testing/helmlite.py — `helm` itself runs in CI) and parsed.

Pins the chart's logic (templates/deployment.yaml, rbac.yaml, _helpers.tpl) and the contract between it
and the controller: every env var it sets is an AppConfig key whose rendered value the config loader
accepts, the leader-election branch adds the Lease Role/RoleBinding, replicas and POD_NAME, the health
port is taken from `healthBindAddress`, and the upstream chart's three ClusterRoles and their bindings
(reference .helm/templates/*) come out with the configured names.
"""
import os

import pytest
import yaml

from ncc.config import AppConfig, load_config
from ncc.testing.helmlite import TemplateError, render, render_chart

CHART = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "deploy", "helm", "nexus-configuration-controller")


def _docs(overrides=None, release=None) -> list:
    out = render_chart(CHART, overrides, release)
    docs = []
    for name, text in out.items():
        for d in yaml.safe_load_all(text):
            if d is not None:
                docs.append(d)
    return docs


def _one(docs, kind):
    found = [d for d in docs if d["kind"] == kind]
    assert len(found) == 1, [d["kind"] for d in docs]
    return found[0]


def _env(deploy) -> dict:
    c = deploy["spec"]["template"]["spec"]["containers"][0]
    return {e["name"]: e.get("value", e.get("valueFrom")) for e in c["env"]}


def test_default_render():
    docs = _docs()
    kinds = sorted(d["kind"] for d in docs)
    assert kinds == ["ClusterRole"] * 3 + ["ClusterRoleBinding"] * 3 + ["Deployment", "ServiceAccount"]
    dep = _one(docs, "Deployment")
    assert dep["spec"]["replicas"] == 1 and dep["spec"]["strategy"]["type"] == "Recreate"
    env = _env(dep)
    assert "NEXUS__LEADER_ELECT" not in env and "POD_NAME" not in env
    assert dep["spec"]["selector"]["matchLabels"].items() <= dep["spec"]["template"]["metadata"]["labels"].items()
    sa = _one(docs, "ServiceAccount")
    assert dep["spec"]["template"]["spec"]["serviceAccountName"] == sa["metadata"]["name"]
    roles = {d["metadata"]["name"]: d for d in docs if d["kind"] == "ClusterRole"}
    assert set(roles) == {f"release-name-nexus-configuration-controller-{s}"
                          for s in ("secret-editor", "configmap-editor", "template-editor")}
    tmpl = roles["release-name-nexus-configuration-controller-template-editor"]
    assert tmpl["rules"][0]["apiGroups"] == ["science.sneaksanddata.com"]
    assert "nexusalgorithmtemplates/status" in tmpl["rules"][0]["resources"]
    assert tmpl["metadata"]["labels"]["rbac.authorization.k8s.io/aggregate-to-edit"] == "true"
    assert "rbac.authorization.k8s.io/aggregate-to-edit" not in \
        roles["release-name-nexus-configuration-controller-secret-editor"]["metadata"]["labels"]
    for b in (d for d in docs if d["kind"] == "ClusterRoleBinding"):
        assert b["roleRef"]["name"] in roles
        assert b["subjects"] == [{"kind": "ServiceAccount", "name": sa["metadata"]["name"], "namespace": "default"}]
    # the volume the shard kubeconfigs come from is mounted where the controller reads them
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["volumeMounts"][0]["mountPath"] == env["NEXUS__SHARD_CONFIG_PATH"]


def test_env_contract_with_the_config_loader():
    """Every NEXUS__* variable is an AppConfig key and the loader accepts every rendered value."""
    env = _env(_one(_docs({"controller": {"leaderElection": {"enabled": True}, "healthBindAddress": ":8081",
                                          "metricsBindAddress": ":9090"}}), "Deployment"))
    nexus = {k: v for k, v in env.items() if k.startswith("NEXUS__")}
    known = {AppConfig.env_of(f) for f in AppConfig.__dataclass_fields__}
    assert set(nexus) <= known, set(nexus) - known
    cfg = load_config(config_dir=None, env=nexus)
    assert cfg.leader_elect is True and cfg.mode == "native" and cfg.health_bind_address == ":8081"
    assert cfg.lease_duration == 15.0 and cfg.renew_deadline == 10.0 and cfg.retry_period == 2.0
    assert cfg.failure_rate_base_delay == 0.03 and cfg.failure_rate_max_delay == 5.0
    assert cfg.client_http2 == "auto"


def test_cpu_affinity_knob():
    """`controller.cpuAffinity` reaches the process as NCC_CPU_AFFINITY (ncc/affinity.py); off by default."""
    env = _env(_one(_docs(), "Deployment"))
    assert env["NCC_CPU_AFFINITY"] == "none" and env["NCC_CPU_AFFINITY_RECHECK_S"] == "30"
    env = _env(_one(_docs({"controller": {"cpuAffinity": "l3", "cpuAffinityRecheckSeconds": 0}}), "Deployment"))
    assert env["NCC_CPU_AFFINITY"] == "l3" and env["NCC_CPU_AFFINITY_RECHECK_S"] == "0"
    from ncc import affinity
    assert affinity.policy_from_env(env["NCC_CPU_AFFINITY"]) == "l3"


def test_leader_election_branch():
    docs = _docs({"controller": {"leaderElection": {"enabled": True, "replicas": 3, "leaseName": "ncc-lease"}}},
                 release={"Namespace": "ops"})
    dep = _one(docs, "Deployment")
    assert dep["spec"]["replicas"] == 3 and dep["spec"]["strategy"]["type"] == "RollingUpdate"
    env = _env(dep)
    assert env["NEXUS__LEADER_ELECT"] == "true" and env["NEXUS__LEADER_ELECTION_LEASE_NAME"] == "ncc-lease"
    assert env["POD_NAME"] == {"fieldRef": {"fieldPath": "metadata.name"}}
    role, binding = _one(docs, "Role"), _one(docs, "RoleBinding")
    assert role["metadata"]["namespace"] == "nexus"  # the Lease lives in the controller namespace
    assert role["rules"][0]["resources"] == ["leases"] and "update" in role["rules"][0]["verbs"]
    assert binding["roleRef"]["name"] == role["metadata"]["name"]
    assert binding["subjects"][0]["namespace"] == "ops"


def test_health_port_datadog_and_extras():
    docs = _docs({"controller": {"healthBindAddress": "0.0.0.0:8086", "datadog": {"enabled": True}},
                  "extraEnv": [{"name": "EXTRA", "value": "1"}], "additionalLabels": {"team": "ml"},
                  "resources": {"limits": {"cpu": "8"}}})
    dep = _one(docs, "Deployment")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["ports"] == [{"name": "health", "containerPort": 8086}]
    assert c["livenessProbe"]["httpGet"] == {"path": "/healthz", "port": "health"}
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    env = _env(dep)
    assert env["DATADOG__API_KEY"] == {"secretKeyRef": {"name": "secretName", "key": "secretKey"}}
    assert env["DD_DOGSTATSD_URL"] == "unix:///var/run/datadog/dsd.socket" and "DD_ENTITY_ID" in env
    assert env["EXTRA"] == "1" and c["resources"] == {"limits": {"cpu": "8"}}
    assert {"name": "dsdsocket", "mountPath": "/var/run/datadog"} in c["volumeMounts"]
    assert dep["metadata"]["labels"]["team"] == "ml"


def test_metrics_port_service_and_service_monitor():
    """ncc extension: `controller.metricsBindAddress` opens a `metrics` container port; `metrics.service` puts
    it behind a Service and `metrics.serviceMonitor` adds a Prometheus-operator ServiceMonitor for it."""
    assert not [d for d in _docs({}) if d["kind"] in ("Service", "ServiceMonitor")]  # off by default
    docs = _docs({"controller": {"metricsBindAddress": ":9090", "healthBindAddress": ":8081"},
                  "metrics": {"service": {"enabled": True},
                              "serviceMonitor": {"enabled": True, "interval": "15s",
                                                 "additionalLabels": {"release": "prom"}}}})
    c = _one(docs, "Deployment")["spec"]["template"]["spec"]["containers"][0]
    assert c["ports"] == [{"name": "health", "containerPort": 8081}, {"name": "metrics", "containerPort": 9090}]
    svc, sm = _one(docs, "Service"), _one(docs, "ServiceMonitor")
    assert svc["spec"]["ports"] == [{"name": "metrics", "port": 9090, "targetPort": "metrics"}]
    dep_labels = _one(docs, "Deployment")["spec"]["selector"]["matchLabels"]
    assert svc["spec"]["selector"] == dep_labels
    assert sm["spec"]["endpoints"] == [{"port": "metrics", "path": "/metrics", "interval": "15s"}]
    assert sm["metadata"]["labels"]["release"] == "prom" and sm["spec"]["selector"]["matchLabels"] == dep_labels
    # the metrics port alone (no health address): ports without probes
    c = _one(_docs({"controller": {"metricsBindAddress": "0.0.0.0:9100", "healthBindAddress": ""}}),
             "Deployment")["spec"]["template"]["spec"]["containers"][0]
    assert c["ports"] == [{"name": "metrics", "containerPort": 9100}] and "livenessProbe" not in c


def test_names_and_switches():
    docs = _docs({"fullnameOverride": "ncc", "serviceAccount": {"create": False, "name": "existing"},
                  "rbac": {"clusterRoleBindings": {"create": False},
                           "clusterRole": {"secretEditor": {"nameOverride": "custom-secrets"},
                                           "configMapEditor": {"create": False}}}})
    assert [d["kind"] for d in docs if d["kind"] == "ServiceAccount"] == []
    assert [d for d in docs if d["kind"] == "ClusterRoleBinding"] == []
    names = sorted(d["metadata"]["name"] for d in docs if d["kind"] == "ClusterRole")
    assert names == ["custom-secrets", "ncc-template-editor"]
    assert _one(docs, "Deployment")["spec"]["template"]["spec"]["serviceAccountName"] == "existing"


def test_template_engine_semantics():
    out = render({"t.yaml": '{{- $x := .Values.a -}}\n{{ if eq $x 1 }}one{{ else if eq $x 2 }}two{{ else }}'
                            'other{{ end }}|{{ range $i, $v := .Values.l }}{{ $i }}={{ $v }},{{ end }}|'
                            '{{ with .Values.missing }}x{{ else }}none{{ end }}|{{ .Values.s | default "d" | quote }}|'
                            '{{ printf "%s-%d" "a" 3 }}|{{ and 1 0 }}{{ or 0 "" "z" }}|{{ dig "p" "q" 7 .Values }}'},
                 {"a": 2, "l": ["x", "y"], "s": ""})
    assert out["t.yaml"] == 'two|0=x,1=y,|none|"d"|a-3|0z|7'
    with pytest.raises(TemplateError):
        render({"t.yaml": "{{ nosuchfunc 1 }}"}, {})
