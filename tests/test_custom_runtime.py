"""examples/custom-runtime: the third-party runtime's own conformance test runs
as part of the suite, plus the cluster-less devroot (OMNIA_CONFIG_DIR)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
EX = os.path.join(HERE, "..", "examples", "custom-runtime")
sys.path.insert(0, os.path.join(EX, "av-preprocessor"))

from conformance_test import (test_converse_reports_frames_for_audio_parts,  # noqa: E402,F401
                              test_example_runtime_is_conformant,
                              test_log_mel_stage_against_numpy_reference)


def test_devroot_config_dir_resolves_like_the_operator(tmp_path, monkeypatch):
    from omnia_amd.runtime.config import RuntimeConfig

    env = {"OMNIA_CONFIG_DIR": os.path.join(EX, "devroot"), "OMNIA_AGENT_NAME": "demo",
           "OMNIA_NAMESPACE": "dev", "OMNIA_PROMPTPACK_PATH": str(tmp_path / "pack.json"),
           "OMNIA_GRPC_PORT": "9100"}
    c = RuntimeConfig.from_env(env)
    assert (c.agent_name, c.namespace, c.grpc_port) == ("demo", "dev", 9100)
    assert c.provider["type"] == "mock" and c.provider["name"] == "demo-mock"
    assert c.promptpack_path == str(tmp_path / "pack.json")
    assert c.context_type == "memory" and c.workspace == "dev-workspace"
    # a real provider's key comes from the devroot Secret, like the in-cluster path
    oa = [p for p in c.extra_providers if p.get("type") == "openai"]
    assert oa and oa[0]["apiKey"] == "sk-devroot-example"


def test_devroot_runtime_serves_a_turn(tmp_path):
    import asyncio
    import json

    from omnia_amd.api.proto import runtime_v1 as pb
    from omnia_amd.runtime import conformance
    from omnia_amd.runtime.app import build_runtime
    from omnia_amd.runtime.config import RuntimeConfig
    from omnia_amd.runtime.server import serve_grpc

    (tmp_path / "pack.json").write_text(json.dumps({
        "id": "d", "name": "d", "version": "1.0.0",
        "template_engine": {"version": "v1", "syntax": "{{variable}}"},
        "prompts": {"default": {"id": "default", "name": "d", "version": "1.0.0",
                                "system_template": "You are terse."}}}))
    env = {"OMNIA_CONFIG_DIR": os.path.join(EX, "devroot"), "OMNIA_AGENT_NAME": "demo",
           "OMNIA_NAMESPACE": "dev", "OMNIA_PROMPTPACK_PATH": str(tmp_path / "pack.json")}

    async def go():
        svc = await build_runtime(RuntimeConfig.from_env(env))
        server, port = await serve_grpc(svc, 0, "127.0.0.1")
        try:
            return await conformance.run(f"127.0.0.1:{port}", 20)
        finally:
            await server.stop(0)

    res = asyncio.run(go())
    assert all(r.passed for r in res), res
