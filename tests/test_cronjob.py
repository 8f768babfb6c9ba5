"""Single-node CronJob controller (LocalLauncher._sync_cronjobs): schedule ->
Job from jobTemplate (owned, deterministic name), concurrencyPolicy Forbid /
Replace, suspend, history limit, status.lastScheduleTime / active."""
from omnia_amd.operator.apistore import APIStore
from omnia_amd.operator.launcher import LocalLauncher

T0 = 1_800_000_000.0  # a minute boundary + 0 s (2027-01-15 08:00:00 UTC)


def _cron(st, policy="Forbid", keep=1, suspend=False):
    st.apply({"apiVersion": "batch/v1", "kind": "CronJob",
              "metadata": {"name": "compact", "namespace": "default"},
              "spec": {"schedule": "*/5 * * * *", "concurrencyPolicy": policy,
                       "suspend": suspend, "successfulJobsHistoryLimit": keep,
                       "jobTemplate": {"metadata": {"labels": {"app": "compaction"}},
                                       "spec": {"template": {"spec": {"containers": [{
                                           "name": "c", "command": ["true"]}]}}}}}})


def _finish(st, name):
    j = st.get("Job", name, "default")
    j["status"] = {"conditions": [{"type": "Complete", "status": "True"}]}
    j["metadata"].pop("resourceVersion", None)
    st.update_status(j)


def test_cronjob_schedules_jobs_with_forbid_and_history():
    st = APIStore()
    _cron(st)
    la = LocalLauncher(st)
    assert la._sync_cronjobs(now=T0) == []  # first sight: the schedule starts here
    made = la._sync_cronjobs(now=T0 + 301)
    assert len(made) == 1
    job = st.get("Job", made[0], "default")
    assert job["metadata"]["labels"] == {"app": "compaction"}
    assert job["metadata"]["ownerReferences"][0]["kind"] == "CronJob"
    assert st.get("CronJob", "compact", "default")["status"]["active"] == [{"name": made[0]}]
    assert la._sync_cronjobs(now=T0 + 700) == []  # Forbid: previous still active
    _finish(st, made[0])
    second = la._sync_cronjobs(now=T0 + 1000)
    assert len(second) == 1 and second != made
    _finish(st, second[0])
    la._sync_cronjobs(now=T0 + 1001)  # history limit 1: the older finished Job goes
    assert st.try_get("Job", made[0], "default") is None
    assert st.try_get("Job", second[0], "default") is not None


def test_cronjob_replace_and_suspend():
    st = APIStore()
    _cron(st, policy="Replace")
    la = LocalLauncher(st)
    la._sync_cronjobs(now=T0)
    first = la._sync_cronjobs(now=T0 + 301)
    second = la._sync_cronjobs(now=T0 + 601)
    assert st.try_get("Job", first[0], "default") is None and second  # replaced
    st2 = APIStore()
    _cron(st2, suspend=True)
    la2 = LocalLauncher(st2)
    la2._sync_cronjobs(now=T0)
    assert la2._sync_cronjobs(now=T0 + 3600) == []
