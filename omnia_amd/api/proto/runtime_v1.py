"""``omnia.runtime.v1`` -- facade <-> runtime contract (Contract-Version 1.3.0).

Field numbers mirror ``api/proto/runtime/v1/runtime.proto:34-443``; field 3 of
ServerMessage stays reserved (the removed ``tool_result``).
"""
from __future__ import annotations

from . import build_file

CONTRACT_VERSION = "1.3.0"  # runtime.proto:10, pkg/runtime/contract/version.go
PACKAGE = "omnia.runtime.v1"
SERVICE = f"{PACKAGE}.RuntimeService"

R = {"repeated": True}

_messages = {
    "ClientMessage": [
        ("session_id", 1, "string"), ("content", 2, "string"),
        ("metadata", 3, ("map", "string", "string")),
        ("parts", 4, "ContentPart", R), ("client_tool_result", 5, "ClientToolResult"),
        ("consent_grants", 6, "string", R), ("duplex_start", 7, "DuplexStart"),
        ("audio_input", 8, "AudioInputChunk"),
    ],
    "ClientToolResult": [
        ("call_id", 1, "string"), ("result_json", 2, "string"), ("is_rejected", 3, "bool"),
        ("rejection_reason", 4, "string"),
    ],
    "ServerMessage": [
        ("chunk", 1, "Chunk", {"oneof": "message"}),
        ("tool_call", 2, "ToolCall", {"oneof": "message"}),
        ("done", 4, "Done", {"oneof": "message"}),
        ("error", 5, "Error", {"oneof": "message"}),
        ("media_chunk", 6, "MediaChunk", {"oneof": "message"}),
        ("interruption", 7, "Interruption", {"oneof": "message"}),
        ("runtime_hello", 8, "RuntimeHello", {"oneof": "message"}),
    ],
    "Chunk": [("content", 1, "string"), ("role", 2, "string")],
    "ToolCall": [
        ("id", 1, "string"), ("name", 2, "string"), ("arguments_json", 3, "string"),
        ("execution", 4, "enum:ToolExecution"), ("consent_message", 5, "string"),
        ("categories", 6, "string", R),
    ],
    "ToolResult": [("id", 1, "string"), ("result_json", 2, "string"), ("is_error", 3, "bool")],
    "Done": [("final_content", 1, "string"), ("usage", 2, "Usage"),
             ("parts", 3, "ContentPart", R)],
    "ContentPart": [("type", 1, "string"), ("text", 2, "string"), ("media", 3, "MediaContent")],
    "MediaContent": [("data", 1, "string"), ("url", 2, "string"), ("mime_type", 3, "string"),
                     ("storage_ref", 4, "string")],
    # field 4 is ours: prompt tokens the engine served from cached KV pages
    "Usage": [("input_tokens", 1, "int32"), ("output_tokens", 2, "int32"),
              ("cost_usd", 3, "float"), ("cached_tokens", 4, "int32")],
    "Error": [("code", 1, "string"), ("message", 2, "string")],
    "Interruption": [],
    "MediaChunk": [("media_id", 1, "string"), ("sequence", 2, "int32"), ("is_last", 3, "bool"),
                   ("mime_type", 4, "string"), ("data", 5, "bytes")],
    "InvocationRequest": [("input_json", 1, "string"), ("invocation_id", 2, "string"),
                          ("metadata", 3, ("map", "string", "string"))],
    "InvocationResponse": [("output_json", 1, "string"), ("usage", 2, "Usage"),
                           ("duration_ms", 3, "int32"), ("invocation_id", 4, "string")],
    "HealthRequest": [],
    "HealthResponse": [("healthy", 1, "bool"), ("status", 2, "string"),
                       ("contract_version", 3, "string"), ("capabilities", 4, "string", R)],
    "HasConversationRequest": [("session_id", 1, "string")],
    "HasConversationResponse": [("state", 1, "enum:ResumeState"), ("detail", 2, "string")],
    "DuplexStart": [("codec", 1, "string"), ("sample_rate", 2, "int32"), ("channels", 3, "int32"),
                    ("system_instruction", 4, "string")],
    "RuntimeHello": [("capabilities", 1, "string", R), ("media", 2, "MediaNegotiation")],
    "MediaNegotiation": [("codec", 1, "string"), ("sample_rate", 2, "int32"),
                         ("channels", 3, "int32"), ("frame_rate", 4, "int32"),
                         ("resolution", 5, "int32")],
    "AudioInputChunk": [("data", 1, "bytes"), ("sequence", 2, "uint32"), ("is_last", 3, "bool")],
}

_enums = {
    "ToolExecution": [("TOOL_EXECUTION_SERVER", 0), ("TOOL_EXECUTION_CLIENT", 1)],
    "ResumeState": [("RESUME_STATE_UNSPECIFIED", 0), ("RESUME_STATE_RESUMABLE", 1),
                    ("RESUME_STATE_NOT_FOUND", 2), ("RESUME_STATE_UNAVAILABLE", 3)],
}

_services = {
    "RuntimeService": {
        "Converse": ("ClientMessage", "ServerMessage", True, True),
        "Invoke": ("InvocationRequest", "InvocationResponse", False, False),
        "Health": ("HealthRequest", "HealthResponse", False, False),
        "HasConversation": ("HasConversationRequest", "HasConversationResponse", False, False),
    }
}

_built = build_file("omnia/runtime/v1/runtime.proto", PACKAGE, _messages, _enums, _services)
FILE_DESCRIPTOR = _built["file"]
M = _built["messages"]

ClientMessage = M["ClientMessage"]
ClientToolResult = M["ClientToolResult"]
ServerMessage = M["ServerMessage"]
Chunk = M["Chunk"]
ToolCall = M["ToolCall"]
ToolResult = M["ToolResult"]
Done = M["Done"]
ContentPart = M["ContentPart"]
MediaContent = M["MediaContent"]
Usage = M["Usage"]
Error = M["Error"]
Interruption = M["Interruption"]
MediaChunk = M["MediaChunk"]
InvocationRequest = M["InvocationRequest"]
InvocationResponse = M["InvocationResponse"]
HealthRequest = M["HealthRequest"]
HealthResponse = M["HealthResponse"]
HasConversationRequest = M["HasConversationRequest"]
HasConversationResponse = M["HasConversationResponse"]
DuplexStart = M["DuplexStart"]
RuntimeHello = M["RuntimeHello"]
MediaNegotiation = M["MediaNegotiation"]
AudioInputChunk = M["AudioInputChunk"]

TOOL_EXECUTION_SERVER = 0
TOOL_EXECUTION_CLIENT = 1
RESUME_STATE_UNSPECIFIED = 0
RESUME_STATE_RESUMABLE = 1
RESUME_STATE_NOT_FOUND = 2
RESUME_STATE_UNAVAILABLE = 3

# capability names (pkg/runtime/contract/*.go)
CAP_INVOKE = "invoke"
CAP_DUPLEX_AUDIO = "duplex_audio"
CAP_CLIENT_TOOLS = "client_tools"
CAP_CONSENT_GRANTS = "consent_grants"
CAP_MEDIA_STORAGE_REF = "media_storage_ref"
CAP_INTERRUPTION = "interruption"
KNOWN_CAPABILITIES = [CAP_INVOKE, CAP_DUPLEX_AUDIO, CAP_CLIENT_TOOLS, CAP_CONSENT_GRANTS,
                      CAP_MEDIA_STORAGE_REF, CAP_INTERRUPTION]

METHOD_CONVERSE = f"/{SERVICE}/Converse"
METHOD_INVOKE = f"/{SERVICE}/Invoke"
METHOD_HEALTH = f"/{SERVICE}/Health"
METHOD_HAS_CONVERSATION = f"/{SERVICE}/HasConversation"
