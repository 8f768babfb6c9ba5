"""Wire-identical protobuf contracts built without protoc.

``omnia.runtime.v1`` mirrors ``api/proto/runtime/v1/runtime.proto`` (Contract-Version
1.3.0) and ``omnia.tools.v1`` mirrors ``api/proto/tools/v1/tools.proto`` field for
field (names, numbers, types, oneof, enums, map entries), so a Go facade built
from the reference's generated stubs talks to our runtime unchanged.  There is
no ``grpcio-tools`` in the image, so the FileDescriptorProtos are assembled
here and registered in a private descriptor pool.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

_TYPES = {
    "string": F.TYPE_STRING, "bytes": F.TYPE_BYTES, "bool": F.TYPE_BOOL, "int32": F.TYPE_INT32,
    "uint32": F.TYPE_UINT32, "int64": F.TYPE_INT64, "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE,
    "uint64": F.TYPE_UINT64, "fixed32": F.TYPE_FIXED32, "fixed64": F.TYPE_FIXED64,
    "sfixed64": F.TYPE_SFIXED64,
}

POOL = descriptor_pool.DescriptorPool()


def _field(msg, name, number, typ, repeated=False, oneof=None, package=""):
    f = msg.field.add()
    f.name = name
    f.number = number
    f.json_name = "".join(w.capitalize() if i else w for i, w in enumerate(name.split("_")))
    f.label = F.LABEL_REPEATED if repeated else F.LABEL_OPTIONAL
    if typ in _TYPES:
        f.type = _TYPES[typ]
    elif typ.startswith("enum:"):
        f.type = F.TYPE_ENUM
        f.type_name = typ[5:] if typ[5:].startswith(".") else f".{package}.{typ[5:]}"
    else:
        f.type = F.TYPE_MESSAGE
        f.type_name = typ if typ.startswith(".") else f".{package}.{typ}"
    if oneof is not None:
        f.oneof_index = oneof
    return f


def build_file(name: str, package: str, messages: dict, enums: dict, services: dict,
               deps: tuple = ()) -> dict:
    """messages: {Msg: [(field, num, type, opts...)]}; map fields as ("map", k, v);
    a type name with a leading "." is fully qualified (another package, listed in
    ``deps`` by file name).  Nested messages are written "Outer.Inner"."""
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = name
    fd.package = package
    fd.syntax = "proto3"
    fd.dependency.extend(deps)
    for ename, values in enums.items():
        e = fd.enum_type.add()
        e.name = ename
        for vname, vnum in values:
            v = e.value.add()
            v.name = vname
            v.number = vnum
    tops: dict = {}
    for mname, fields in messages.items():
        if "." in mname:  # nested message (declared after its parent)
            outer, inner = mname.split(".", 1)
            m = tops[outer].nested_type.add()
            m.name = inner
        else:
            m = fd.message_type.add()
            m.name = mname
            tops[mname] = m
        oneofs: dict[str, int] = {}
        for spec in fields:
            fname, num, typ = spec[0], spec[1], spec[2]
            opts = spec[3] if len(spec) > 3 else {}
            if isinstance(typ, tuple) and typ[0] == "map":
                entry = m.nested_type.add()
                entry.name = "".join(w.capitalize() for w in fname.split("_")) + "Entry"
                entry.options.map_entry = True
                _field(entry, "key", 1, typ[1], package=package)
                _field(entry, "value", 2, typ[2], package=package)
                _field(m, fname, num, f".{package}.{mname}.{entry.name}", repeated=True,
                       package=package)
                continue
            oneof = None
            if "oneof" in opts:
                if opts["oneof"] not in oneofs:
                    oneofs[opts["oneof"]] = len(m.oneof_decl)
                    m.oneof_decl.add().name = opts["oneof"]
                oneof = oneofs[opts["oneof"]]
            _field(m, fname, num, typ, repeated=opts.get("repeated", False), oneof=oneof,
                   package=package)
    for sname, methods in services.items():
        s = fd.service.add()
        s.name = sname
        for mname, (inp, out, cs, ss) in methods.items():
            mm = s.method.add()
            mm.name = mname
            mm.input_type = f".{package}.{inp}"
            mm.output_type = f".{package}.{out}"
            mm.client_streaming = cs
            mm.server_streaming = ss
    POOL.Add(fd)
    classes = {}
    for mname in messages:
        classes[mname] = message_factory.GetMessageClass(
            POOL.FindMessageTypeByName(f"{package}.{mname}"))
    enum_objs = {e: POOL.FindEnumTypeByName(f"{package}.{e}") for e in enums}
    return {"messages": classes, "enums": enum_objs, "file": fd}
