"""Chat message model, Llama-3 chat template and tool-call parsing.

The reference hands message lists to PromptKit which speaks each vendor's chat
API.  The in-node engine needs the model's own chat template instead: we render
Llama-3 headers (``<|start_header_id|>role<|end_header_id|>`` ... ``<|eot_id|>``),
expose tools in the Llama-3.1 JSON tool-calling convention, and parse tool calls
back out of generated text (``{"name": ..., "parameters": {...}}`` objects,
optionally after ``<|python_tag|>``).
"""
from __future__ import annotations

import json
import re
import uuid
from dataclasses import asdict, dataclass, field


@dataclass
class ToolCallReq:
    id: str
    name: str
    arguments: dict

    @property
    def arguments_json(self) -> str:
        return json.dumps(self.arguments, separators=(",", ":"))


@dataclass
class Message:
    role: str  # system | user | assistant | tool
    content: str = ""
    tool_calls: list = field(default_factory=list)  # list[ToolCallReq] (assistant)
    tool_call_id: str = ""  # (tool)
    name: str = ""  # tool name (tool)
    parts: list = field(default_factory=list)  # multimodal parts (dicts)

    def to_dict(self) -> dict:
        d = {"role": self.role, "content": self.content}
        if self.tool_calls:
            d["tool_calls"] = [asdict(t) for t in self.tool_calls]
        if self.tool_call_id:
            d["tool_call_id"] = self.tool_call_id
        if self.name:
            d["name"] = self.name
        if self.parts:
            d["parts"] = self.parts
        return d

    @staticmethod
    def from_dict(d: dict) -> "Message":
        return Message(role=d["role"], content=d.get("content", ""),
                       tool_calls=[ToolCallReq(**t) for t in d.get("tool_calls", [])],
                       tool_call_id=d.get("tool_call_id", ""), name=d.get("name", ""),
                       parts=d.get("parts", []))


def render_llama3(messages: list[Message], tools: list[dict] | None = None,
                  add_generation_prompt: bool = True) -> str:
    out = ["<|begin_of_text|>"]
    sys_extra = ""
    if tools:
        sys_extra = (
            "\n\nYou have access to the following functions. To call a function, respond with "
            "a JSON object {\"name\": function name, \"parameters\": dictionary of argument "
            "name and its value}. Do not use variables.\n\n"
            + "\n\n".join(json.dumps({"type": "function", "function": t}) for t in tools))
    first_system = True
    for m in messages:
        role = m.role
        content = m.content
        if role == "system" and first_system:
            content = content + sys_extra
            first_system = False
        if role == "assistant" and m.tool_calls:
            content = content + "".join(
                json.dumps({"name": t.name, "parameters": t.arguments}) for t in m.tool_calls)
        if role == "tool":
            role = "ipython"
        out.append(f"<|start_header_id|>{role}<|end_header_id|>\n\n{content}<|eot_id|>")
    if first_system and sys_extra:
        out.insert(1, f"<|start_header_id|>system<|end_header_id|>\n\n{sys_extra.strip()}"
                      "<|eot_id|>")
    if add_generation_prompt:
        out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(out)


def shared_prefix_len(messages: list[Message], tools: list[dict] | None, encode,
                      prompt_ids: list[int]) -> int:
    """Leading tokens of ``prompt_ids`` that render the conversation's leading
    system message(s) and the tool schemas -- the deployment's PromptPack prefix,
    the only part of a prompt the engine may publish for cross-session KV sharing
    (``SamplingParams.share_limit``; engine/kv_manager.py).  A user's own turns
    never fall inside it."""
    head = []
    for m in messages:
        if m.role != "system":
            break
        head.append(m)
    if not head and not tools:
        return 0
    ids = encode(render_llama3(head, tools or None, add_generation_prompt=False))
    n = min(len(ids), len(prompt_ids))
    i = 0
    while i < n and ids[i] == prompt_ids[i]:
        i += 1
    return i


_JSON_OBJ = re.compile(r"\{.*\}", re.S)


def parse_tool_calls(text: str, tool_names: set[str]) -> tuple[str, list[ToolCallReq]]:
    """Extract Llama-3 style tool calls.  Returns (remaining_text, calls)."""
    if not tool_names:
        return text, []
    body = text.replace("<|python_tag|>", "").strip()
    calls: list[ToolCallReq] = []
    # one or more JSON objects, possibly separated by ';' or newlines
    dec = json.JSONDecoder()
    i = 0
    rest = []
    while i < len(body):
        j = body.find("{", i)
        if j < 0:
            rest.append(body[i:])
            break
        rest.append(body[i:j])
        try:
            obj, end = dec.raw_decode(body, j)
        except (json.JSONDecodeError, RecursionError):  # model output: garbage or deep nesting
            rest.append(body[j:])
            break
        name = obj.get("name") if isinstance(obj, dict) else None
        if isinstance(name, str) and name in tool_names:
            args = obj.get("parameters", obj.get("arguments", {}))
            if isinstance(args, str):
                try:
                    args = json.loads(args)
                except (json.JSONDecodeError, RecursionError):
                    args = {"input": args}
            calls.append(ToolCallReq(id="call_" + uuid.uuid4().hex[:12], name=obj["name"],
                                     arguments=args if isinstance(args, dict) else {}))
        else:
            rest.append(body[j:end])
        i = end
    if not calls:
        return text, []
    return "".join(rest).strip(" ;\n"), calls
