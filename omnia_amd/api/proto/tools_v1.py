"""``omnia.tools.v1`` -- external tool service contract (``api/proto/tools/v1/tools.proto:12-66``)."""
from __future__ import annotations

from . import build_file

PACKAGE = "omnia.tools.v1"
SERVICE = f"{PACKAGE}.ToolService"

_messages = {
    "ToolRequest": [("tool_name", 1, "string"), ("arguments_json", 2, "string"),
                    ("metadata", 3, ("map", "string", "string"))],
    "ToolResponse": [("result_json", 1, "string"), ("is_error", 2, "bool"),
                     ("error_message", 3, "string")],
    "ListToolsRequest": [],
    "ListToolsResponse": [("tools", 1, "ToolInfo", {"repeated": True})],
    "ToolInfo": [("name", 1, "string"), ("description", 2, "string"),
                 ("input_schema", 3, "string")],
}
_services = {"ToolService": {
    "Execute": ("ToolRequest", "ToolResponse", False, False),
    "ListTools": ("ListToolsRequest", "ListToolsResponse", False, False),
}}

_built = build_file("omnia/tools/v1/tools.proto", PACKAGE, _messages, {}, _services)
M = _built["messages"]
ToolRequest = M["ToolRequest"]
ToolResponse = M["ToolResponse"]
ListToolsRequest = M["ListToolsRequest"]
ListToolsResponse = M["ListToolsResponse"]
ToolInfo = M["ToolInfo"]

METHOD_EXECUTE = f"/{SERVICE}/Execute"
METHOD_LIST_TOOLS = f"/{SERVICE}/ListTools"
