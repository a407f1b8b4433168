"""acl.SubjectTree / Subject message classes built at run time from a descriptor that restates
proto/ory/keto/acl/v1alpha1/acl.proto and expand_service.proto (field numbers and types only), so
the tests can serialize the oracle's trees with the protobuf runtime and compare bytes with the
engine's encoder (keto_tree_proto).  Test infrastructure only."""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto


def _classes():
    fd = descriptor_pb2.FileDescriptorProto(name="keto_acl_restated.proto", package="ory.keto.acl.v1alpha1",
                                            syntax="proto3")
    ss = fd.message_type.add(name="SubjectSet")
    for i, n in enumerate(("namespace", "object", "relation"), 1):
        ss.field.add(name=n, number=i, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
    sub = fd.message_type.add(name="Subject")
    sub.oneof_decl.add(name="ref")
    sub.field.add(name="id", number=1, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL, oneof_index=0)
    sub.field.add(name="set", number=2, type=_F.TYPE_MESSAGE, label=_F.LABEL_OPTIONAL, oneof_index=0,
                  type_name=".ory.keto.acl.v1alpha1.SubjectSet")
    en = fd.enum_type.add(name="NodeType")
    for n, v in (("NODE_TYPE_UNSPECIFIED", 0), ("NODE_TYPE_UNION", 1), ("NODE_TYPE_EXCLUSION", 2),
                 ("NODE_TYPE_INTERSECTION", 3), ("NODE_TYPE_LEAF", 4)):
        en.value.add(name=n, number=v)
    st = fd.message_type.add(name="SubjectTree")
    st.field.add(name="node_type", number=1, type=_F.TYPE_ENUM, label=_F.LABEL_OPTIONAL,
                 type_name=".ory.keto.acl.v1alpha1.NodeType")
    st.field.add(name="subject", number=2, type=_F.TYPE_MESSAGE, label=_F.LABEL_OPTIONAL,
                 type_name=".ory.keto.acl.v1alpha1.Subject")
    st.field.add(name="children", number=3, type=_F.TYPE_MESSAGE, label=_F.LABEL_REPEATED,
                 type_name=".ory.keto.acl.v1alpha1.SubjectTree")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = getattr(message_factory, "GetMessageClass", None)
    if get is None:
        f = message_factory.MessageFactory(pool)
        get = lambda d: f.GetPrototype(d)
    return get(pool.FindMessageTypeByName("ory.keto.acl.v1alpha1.SubjectTree"))


SubjectTree = _classes()


def tree_json_to_proto(js) -> bytes:
    """Tree.ToProto() (internal/expand/tree.go:165-188) of a reference JSON tree, serialized."""
    def fill(m, t):
        m.node_type = 4 if t["type"] == "leaf" else 1
        if "subject_id" in t:
            m.subject.id = t["subject_id"]
        else:
            s = t["subject_set"]
            m.subject.set.SetInParent()
            m.subject.set.namespace = s["namespace"]
            m.subject.set.object = s["object"]
            m.subject.set.relation = s["relation"]
        if t["type"] != "leaf":
            for c in t.get("children", []) or []:
                fill(m.children.add(), c)
    m = SubjectTree()
    fill(m, js)
    return m.SerializeToString(deterministic=True)
