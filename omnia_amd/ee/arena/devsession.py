"""ArenaDevSession reconciler (``ee/internal/controller/arenadevsession_controller.go``).

A dev session is an interactive arena console (``ee/dev_console.py``: the
WebSocket console the PromptKit LSP / dashboard drive) run for one user in one
workspace namespace.  State machine, as in the reference:

``"" -> Pending -> Starting -> Ready [-> Stopping -> Stopped] | Failed``

* a finalizer is added first (cleanup must run before the object goes);
* **Starting** creates, owned by the session: a ServiceAccount, a Role that may
  read arena sources / config maps / providers / tool registries / secrets, its
  RoleBinding, a Deployment running the console (image + ``--port 8080``,
  POD_NAMESPACE / OMNIA_WORKSPACE_NAME / provider credentials from the
  namespace's Providers' ``secretRef`` as env, ``/healthz`` probes, requests /
  limits, ``podOverrides``) and a Service -- all named ``adc-<name>`` (names over
  63 characters are truncated and suffixed with 8 hex of their sha256);
* **Ready** once the Deployment reports a ready replica: ``startedAt``,
  ``lastActivityAt``, ``serviceName`` and ``endpoint`` =
  ``ws://adc-<name>.<ns>.svc:8080/ws`` (plus the local endpoint the launcher
  bound, in single-node mode);
* **idle timeout**: a Ready session whose ``lastActivityAt`` is older than
  ``spec.idleTimeout`` (Go duration, default 30m) is stopped -- the console
  reports activity with the ``omnia.altairalabs.ai/last-activity`` annotation
  (RFC 3339), which the reconciler folds into ``status.lastActivityAt``;
* **Stopping** deletes the five resources and ends in **Stopped** with an empty
  endpoint; deleting the session runs the same cleanup, then drops the
  finalizer.
"""
from __future__ import annotations

import hashlib
import logging
import time

from ...operator.apistore import owner_ref, set_condition

log = logging.getLogger("omnia.arena.devsession")

FINALIZER = "omnia.altairalabs.ai/arenadevsession-cleanup"
ACTIVITY_ANNOTATION = "omnia.altairalabs.ai/last-activity"
DEFAULT_IDLE_S = 30 * 60.0
DEFAULT_IMAGE = "ghcr.io/altairalabs/omnia-arena-dev-console:latest"
CONSOLE_CMD = ["python", "-m", "omnia_amd.ee.dev_console"]
LABEL_COMPONENT = "omnia.altairalabs.ai/component"


def resource_name(name: str) -> str:
    full = "adc-" + name
    if len(full) <= 63:
        return full
    h = hashlib.sha256(name.encode()).hexdigest()[:8]
    return f"adc-{name[:50]}-{h}"


def _ts(t: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def _parse_ts(v) -> float | None:
    if not v:
        return None
    import calendar

    try:
        return float(calendar.timegm(time.strptime(str(v)[:19], "%Y-%m-%dT%H:%M:%S")))
    except ValueError:
        return None


def _duration(s: str | None, default: float) -> float:
    if not s:
        return default
    from ...utils.cron import CronError, _duration as dur

    try:
        return dur(s)
    except CronError:
        return default


class ArenaDevSessionReconciler:
    kind = "ArenaDevSession"

    def __init__(self, image: str = DEFAULT_IMAGE, service_account: str = "",
                 now=time.time):
        self.image = image
        self.service_account = service_account  # workspace runtime SA: nothing to create
        self.now = now

    # ------------------------------------------------------------------ loop
    def reconcile(self, store, ns, name):
        ns = ns or "default"
        s = store.try_get(self.kind, name, ns)
        if s is None:
            return None
        md = s["metadata"]
        if md.get("deletionTimestamp"):
            return self._delete(store, s)
        if FINALIZER not in (md.get("finalizers") or []):
            md.setdefault("finalizers", []).append(FINALIZER)
            s.pop("status", None)
            store.update(s)
            return 1.0
        st = dict(s.get("status") or {})
        if not st.get("phase"):
            st["phase"] = "Pending"
        act = _parse_ts((md.get("annotations") or {}).get(ACTIVITY_ANNOTATION))
        if act and act > (_parse_ts(st.get("lastActivityAt")) or 0):
            st["lastActivityAt"] = _ts(act)
        s["status"] = st
        if self._idle(s):
            log.info("stopping idle dev session %s/%s", ns, name)
            return self._cleanup(store, s, reason="IdleTimeout")
        phase = st["phase"]
        if phase == "Pending":
            return self._start(store, s)
        if phase == "Starting":
            return self._wait_ready(store, s)
        if phase == "Ready":
            store.update_status(s)
            return 60.0
        if phase == "Stopping":
            return self._cleanup(store, s)
        store.update_status(s)
        return None

    def _idle(self, s) -> bool:
        st = s["status"]
        if st.get("phase") != "Ready":
            return False
        last = _parse_ts(st.get("lastActivityAt"))
        if last is None:
            return False
        return self.now() - last > _duration(s["spec"].get("idleTimeout"), DEFAULT_IDLE_S)

    # ------------------------------------------------------------------ phases
    def _start(self, store, s):
        st = s["status"]
        st.update(phase="Starting", message="Creating dev console resources")
        store.update_status(s)
        step = "ServiceAccount"
        try:
            ns, rn, own = s["metadata"]["namespace"], resource_name(s["metadata"]["name"]), \
                [owner_ref(s)]
            labels = self._labels(s)
            sa = self.service_account or rn
            if not self.service_account:
                store.apply({"apiVersion": "v1", "kind": "ServiceAccount",
                             "metadata": {"name": rn, "namespace": ns, "labels": labels,
                                          "ownerReferences": own}})
            step = "Role"
            store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                         "metadata": {"name": rn, "namespace": ns, "labels": labels,
                                      "ownerReferences": own},
                         "rules": [
                             {"apiGroups": ["omnia.altairalabs.ai"],
                              "resources": ["arenasources", "arenajobs", "providers",
                                            "toolregistries"],
                              "verbs": ["get", "list", "watch"]},
                             {"apiGroups": [""], "resources": ["secrets"], "verbs": ["get"]},
                             {"apiGroups": [""], "resources": ["configmaps"],
                              "verbs": ["get", "list"]}]})
            step = "RoleBinding"
            store.apply({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                         "metadata": {"name": rn, "namespace": ns, "labels": labels,
                                      "ownerReferences": own},
                         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role",
                                     "name": rn},
                         "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": ns}]})
            step = "Deployment"
            store.apply(self._deployment(store, s, rn, sa, labels, own))
            step = "Service"
            store.apply({"apiVersion": "v1", "kind": "Service",
                         "metadata": {"name": rn, "namespace": ns, "labels": labels,
                                      "ownerReferences": own},
                         "spec": {"selector": {"app": rn},
                                  "ports": [{"name": "http", "port": 8080,
                                             "targetPort": "http"}]}})
        except Exception as e:  # noqa: BLE001 - admission / API errors
            return self._failed(store, s, f"Failed to create {step}", e)
        return 2.0

    def _deployment(self, store, s, rn, sa, labels, own) -> dict:
        spec, ns = s["spec"], s["metadata"]["namespace"]
        env = [{"name": "POD_NAMESPACE", "value": ns},
               {"name": "OMNIA_DEV_SESSION", "value": s["metadata"]["name"]},
               {"name": "OMNIA_ARENA_PROJECT", "value": spec.get("projectId", "")}]
        if spec.get("workspace"):
            env.append({"name": "OMNIA_WORKSPACE_NAME", "value": spec["workspace"]})
        env += self._provider_env(store, ns)
        res = spec.get("resources") or {}
        container = {
            "name": "arena-dev-console", "image": spec.get("image") or self.image,
            "imagePullPolicy": "IfNotPresent", "command": list(CONSOLE_CMD),
            "args": ["--port", "8080"],
            "ports": [{"name": "http", "containerPort": 8080, "protocol": "TCP"}],
            "env": env,
            "readinessProbe": {"httpGet": {"path": "/healthz", "port": 8080},
                               "periodSeconds": 5},
            "livenessProbe": {"httpGet": {"path": "/healthz", "port": 8080},
                              "periodSeconds": 20},
            "resources": {"requests": res.get("requests") or {"cpu": "100m",
                                                              "memory": "256Mi"},
                          "limits": res.get("limits") or {"cpu": "1", "memory": "1Gi"}},
            "volumeMounts": [{"name": "tmp", "mountPath": "/tmp"}],
            "securityContext": {"runAsNonRoot": True, "readOnlyRootFilesystem": True,
                                "allowPrivilegeEscalation": False},
        }
        pod = {"serviceAccountName": sa, "containers": [container],
               "volumes": [{"name": "tmp", "emptyDir": {}}]}
        tmeta = {"labels": {**labels, "app": rn}}
        po = spec.get("podOverrides") or {}
        for k in ("nodeSelector", "tolerations", "affinity", "priorityClassName",
                  "imagePullSecrets"):
            if po.get(k):
                pod[k] = po[k]
        if po.get("labels"):
            tmeta["labels"].update(po["labels"])
        if po.get("annotations"):
            tmeta["annotations"] = dict(po["annotations"])
        if po.get("env"):
            container["env"] = container["env"] + list(po["env"])
        return {"apiVersion": "apps/v1", "kind": "Deployment",
                "metadata": {"name": rn, "namespace": ns,
                             "labels": {**labels, LABEL_COMPONENT: "arena-dev-console"},
                             "ownerReferences": own},
                "spec": {"replicas": 1, "selector": {"matchLabels": {"app": rn}},
                         "template": {"metadata": tmeta, "spec": pod}}}

    @staticmethod
    def _provider_env(store, ns) -> list[dict]:
        """Credentials of the namespace's Providers as env vars referencing their
        secrets (``buildProviderEnvVars``): ``<PROVIDER>_API_KEY``."""
        out, seen = [], set()
        for p in store.list("Provider", ns):
            ref = ((p.get("spec") or {}).get("credential") or {}).get("secretRef") or \
                (p.get("spec") or {}).get("secretRef") or {}
            if not ref.get("name"):
                continue
            var = (p["spec"].get("type") or p["metadata"]["name"]).upper().replace("-", "_") + \
                "_API_KEY"
            if var in seen:
                continue
            seen.add(var)
            out.append({"name": var, "valueFrom": {"secretKeyRef": {
                "name": ref["name"], "key": ref.get("key") or "api-key", "optional": True}}})
        return out

    @staticmethod
    def _labels(s) -> dict:
        return {"app.kubernetes.io/name": "arena-dev-console",
                "app.kubernetes.io/instance": s["metadata"]["name"],
                "app.kubernetes.io/managed-by": "omnia-arena-controller",
                "omnia.altairalabs.ai/dev-session": s["metadata"]["name"]}

    def _wait_ready(self, store, s):
        ns, rn = s["metadata"]["namespace"], resource_name(s["metadata"]["name"])
        dep = store.try_get("Deployment", rn, ns)
        st = s["status"]
        if dep is not None and (dep.get("status") or {}).get("readyReplicas", 0) > 0:
            now = _ts(self.now())
            st.update(phase="Ready", startedAt=now, lastActivityAt=now, serviceName=rn,
                      endpoint=f"ws://{rn}.{ns}.svc:8080/ws", message="Dev console is ready")
            svc = store.try_get("Service", rn, ns)
            local = ((svc or {}).get("status") or {}).get("endpoint")
            if local:
                host = local.split("://", 1)[-1].rstrip("/")
                st["localEndpoint"] = f"ws://{host}/ws"
            set_condition(st, "Ready", True, "DeploymentReady", "Dev console deployment is ready")
            store.update_status(s)
            return 60.0
        st["message"] = "Waiting for dev console to start"
        store.update_status(s)
        return 2.0

    def _cleanup(self, store, s, reason: str = "Stopping"):
        st = s["status"]
        if st.get("phase") != "Stopping":
            st.update(phase="Stopping", message=f"Cleaning up dev console ({reason})")
            store.update_status(s)
            s = store.get(self.kind, s["metadata"]["name"], s["metadata"]["namespace"])
            st = s["status"]
        ns, rn = s["metadata"]["namespace"], resource_name(s["metadata"]["name"])
        kinds = ["Deployment", "Service", "RoleBinding", "Role"]
        if not self.service_account:
            kinds.append("ServiceAccount")
        for kind in kinds:
            try:
                store.delete(kind, rn, ns)
            except KeyError:
                pass
            except Exception as e:  # noqa: BLE001
                if type(e).__name__ != "NotFound":
                    return self._failed(store, s, f"Failed to delete {kind}", e)
        st.update(phase="Stopped", endpoint="", message="Dev console stopped")
        st.pop("localEndpoint", None)
        set_condition(st, "Ready", False, reason, "Dev console stopped")
        store.update_status(s)
        return None

    def _delete(self, store, s):
        if (s.get("status") or {}).get("phase") != "Stopped":
            s["status"] = dict(s.get("status") or {})
            self._cleanup(store, s, reason="Deleted")
            s = store.try_get(self.kind, s["metadata"]["name"], s["metadata"]["namespace"])
            if s is None:
                return None
        fins = [f for f in s["metadata"].get("finalizers") or [] if f != FINALIZER]
        s["metadata"]["finalizers"] = fins
        s.pop("status", None)
        store.update(s)
        return None

    def _failed(self, store, s, msg: str, err: Exception):
        st = s["status"]
        st.update(phase="Failed", message=f"{msg}: {err}")
        set_condition(st, "Ready", False, "Failed", f"{msg}: {err}")
        store.update_status(s)
        return None
