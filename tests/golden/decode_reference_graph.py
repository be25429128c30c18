"""Extract the Q-net definition facts from the reference's compiled Keras graphs -> tests/golden/*_graph_facts.json.

Generator for a data fixture (run here, where /root/reference exists; the GPU box never reads the reference):

    python tests/golden/decode_reference_graph.py [/root/reference]

Inputs (reference files, read as data, nothing in them is executed):
  src/ql-with-tensorflow/python_model/saved/<model>/saved_model.pb   SavedModel protobuf: the `train_model`,
      `batch_predict_max_future_reward` and `predict_action` FunctionDefs (create_ql_model_breakout_84x84x4_3_32.py:35-82
      traced by TF 2.12), node ops / inputs / attributes / inferred output shapes
  src/ql-with-tensorflow/python_model/saved/<model>/keras_metadata.pb   the Keras training_config JSON (loss class and
      delta, optimizer class and its float32 hyperparameters)

The protobuf is decoded by a small wire-format reader (varint / fixed / length-delimited records) with the field numbers
of TensorFlow's published schemas (saved_model.proto, meta_graph.proto, graph.proto, function.proto, node_def.proto,
attr_value.proto, tensor.proto, tensor_shape.proto, op_def.proto); no TensorFlow or generated classes are needed.
"""
import json
import os
import struct
import sys

DTYPES = {1: "float32", 2: "float64", 3: "int32", 4: "uint8", 7: "string", 9: "int64", 10: "bool", 20: "resource"}


# ---------------- protobuf wire format ----------------
def _varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def records(b):
    """[(field, wire_type, value)]: value = int (varint), bytes (length-delimited / fixed32 / fixed64)"""
    out, i = [], 0
    while i < len(b):
        key, i = _varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 2:
            n, i = _varint(b, i)
            v, i = b[i:i + n], i + n
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"wire type {wt}")
        out.append((f, wt, v))
    return out


def first(recs, field):
    for f, _, v in recs:
        if f == field:
            return v
    return None


def every(recs, field):
    return [v for f, _, v in recs if f == field]


def _signed(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def _packed_varints(v, wt):
    if wt != 2:
        return [_signed(v)]
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(_signed(x))
    return out


def shape_proto(b):   # TensorShapeProto: dim = 2 (Dim: size = 1), unknown_rank = 3
    recs = records(b)
    if first(recs, 3):
        return None
    return [_signed(first(records(d), 1) or 0) for d in every(recs, 2)]


def tensor_proto(b):   # TensorProto: dtype 1, tensor_shape 2, tensor_content 4, float_val 5, int_val 7, int64_val 10
    recs = records(b)
    dt = DTYPES.get(first(recs, 1))
    out = {"dtype": dt, "shape": shape_proto(first(recs, 2) or b"")}
    content = first(recs, 4)
    vals = []
    if content is not None:
        fmt = {"float32": "f", "int32": "i", "int64": "q"}.get(dt)
        if fmt:
            vals = list(struct.unpack("<%d%s" % (len(content) // struct.calcsize(fmt), fmt), content))
    for f, wt, v in recs:
        if f == 5:
            vals += list(struct.unpack("<%df" % (len(v) // 4), v))
        elif f in (7, 10):
            vals += _packed_varints(v, wt)
    out["values"] = vals
    return out


def attr_value(b):   # AttrValue oneof: list 1, s 2, i 3, f 4, b 5, type 6, shape 7, tensor 8, func 10
    for f, wt, v in records(b):
        if f == 2:
            return v.decode("utf-8", "replace")
        if f == 3:
            return _signed(v)
        if f == 4:
            return struct.unpack("<f", v)[0]
        if f == 5:
            return bool(v)
        if f == 6:
            return DTYPES.get(v, v)
        if f == 7:
            return {"shape": shape_proto(v)}
        if f == 8:
            return {"tensor": tensor_proto(v)}
        if f == 10:
            return {"func": first(records(v), 1).decode()}
        if f == 1:   # ListValue: s 2, i 3, f 4, type 6, shape 7
            lst = []
            for g, wt2, w in records(v):
                if g == 2:
                    lst.append(w.decode("utf-8", "replace"))
                elif g == 3:
                    lst += _packed_varints(w, wt2)
                elif g == 4:
                    lst += list(struct.unpack("<%df" % (len(w) // 4), w))
                elif g == 6:
                    lst += [DTYPES.get(x, x) for x in _packed_varints(w, wt2)]
                elif g == 7:
                    lst.append(shape_proto(w))
            return lst
    return None


def node_def(b):   # NodeDef: name 1, op 2, input 3, attr 5 (map<string, AttrValue>)
    recs = records(b)
    attrs = {}
    for entry in every(recs, 5):
        er = records(entry)
        attrs[first(er, 1).decode()] = attr_value(first(er, 2) or b"")
    return {"name": first(recs, 1).decode(), "op": first(recs, 2).decode(),
            "input": [x.decode() for x in every(recs, 3)], "attr": attrs}


def functions(saved_model_pb):
    """SavedModel (meta_graphs 2) -> MetaGraphDef (graph_def 2) -> GraphDef (library 2) -> FunctionDef (function 1):
    {name: {"inputs": [(name, dtype)], "nodes": [NodeDef]}}; FunctionDef: signature 1 (OpDef: name 1, input_arg 2
    (ArgDef: name 1, type 3)), node_def 3"""
    mg = first(records(saved_model_pb), 2)
    gd = first(records(mg), 2)
    lib = first(records(gd), 2)
    out = {}
    for fn in every(records(lib), 1):
        fr = records(fn)
        sig = records(first(fr, 1))
        args = [(first(records(a), 1).decode(), DTYPES.get(first(records(a), 3))) for a in every(sig, 2)]
        out[first(sig, 1).decode()] = {"inputs": args, "nodes": [node_def(n) for n in every(fr, 3)]}
    return out


def keras_training_config(keras_metadata_pb):
    """keras_metadata.pb: SavedMetadata of SavedObject records whose metadata field is the Keras JSON; the model's
    record holds "training_config"."""
    for f, _, v in records(keras_metadata_pb):
        if f != 1:
            continue
        for g, _, w in records(v):
            if g == 5 and b"training_config" in w:
                return json.loads(w.decode())["training_config"]
    raise ValueError("no training_config in keras_metadata.pb")


# ---------------- facts ----------------
def _fn(fns, key):
    names = [n for n in fns if key in n]
    assert len(names) == 1, (key, names)
    return fns[names[0]]


def _out_shape(node):
    s = node["attr"].get("_output_shapes")
    return s[0] if s else None


def _const(nodes, name):
    n = [x for x in nodes if x["name"] == name]
    assert len(n) == 1, name
    return n[0]["attr"]["value"]["tensor"]["values"]


def facts(model_dir):
    fns = functions(open(os.path.join(model_dir, "saved_model.pb"), "rb").read())
    tc = keras_training_config(open(os.path.join(model_dir, "keras_metadata.pb"), "rb").read())
    tm = _fn(fns, "_train_model_")
    nodes = tm["nodes"]
    by_op = {}
    for n in nodes:
        by_op.setdefault(n["op"], []).append(n)
    conv_fwd = [{"layer": n["name"].split("/")[1], "strides": n["attr"]["strides"], "padding": n["attr"]["padding"],
                 "data_format": n["attr"].get("data_format", "NHWC"),
                 "dilations": n["attr"].get("dilations", [1, 1, 1, 1]), "output_shape": _out_shape(n)}
                for n in by_op.get("Conv2D", [])]
    conv_bwd = sorted({(n["op"], tuple(n["attr"]["strides"]), n["attr"]["padding"]) for n in nodes
                       if n["op"] in ("Conv2DBackpropInput", "Conv2DBackpropFilter")})
    matmuls = [{"name": n["name"], "transpose_a": bool(n["attr"].get("transpose_a", False)),
                "transpose_b": bool(n["attr"].get("transpose_b", False)), "output_shape": _out_shape(n)}
               for n in by_op.get("MatMul", [])]
    adam = by_op.get("ResourceApplyAdam", [])
    clip_nodes = [n for n in nodes if n["name"].startswith("Adam/clip_by_norm") and n["op"] == "Maximum"]
    f = {
        "signature_inputs": [a for a in tm["inputs"] if a[1] != "resource"],
        "input_shapes": {n["name"]: _out_shape(n) for n in nodes if n["name"] in ("one_hot",)},
        "conv2d_forward": conv_fwd,
        "conv2d_backward": [list(x) for x in conv_bwd],
        "flatten_shape": _const(nodes, [n["name"] for n in nodes if n["name"].endswith("flatten/Const")][0]),
        "matmul": matmuls,
        "relu_count": len(by_op.get("Relu", [])),
        "optimizer_config": tc["optimizer_config"],
        "loss_config": tc["loss"],
        "clip_by_norm": {"count": len(clip_nodes),
                         "clip_norms": [_const(nodes, n["input"][1].split(":")[0])[0] for n in clip_nodes],
                         "ops": sorted({n["op"] for n in nodes if n["name"].startswith("Adam/clip_by_norm/")})},
        "resource_apply_adam": {"count": len(adam),
                                "use_locking": sorted({bool(n["attr"].get("use_locking", False)) for n in adam}),
                                "use_nesterov": sorted({bool(n["attr"].get("use_nesterov", False)) for n in adam}),
                                "inputs_after_slots": sorted({tuple(x.split(":")[0] for x in n["input"][3:9]) for n in adam}),
                                "variables": [n["input"][0] for n in adam]},
        "adam_epsilon_const": _const(nodes, "Adam/Const")[0],
        "beta_power": [n["op"] for n in nodes if n["name"] in ("Adam/Pow", "Adam/Pow_1")],
    }
    if any(n["name"].startswith("huber_loss/") for n in nodes):
        f["loss"] = {
            "kind": "huber",
            "delta": _const(nodes, "huber_loss/Cast/x")[0],
            "half": _const(nodes, "huber_loss/Const")[0],
            "quadratic_branch": [n["op"] for n in nodes if n["name"] in ("huber_loss/Square", "huber_loss/mul")],
            "elementwise_shape": _out_shape([n for n in nodes if n["name"] == "huber_loss/Sub"][0]),
            "mean_axis": _const(nodes, "huber_loss/Mean/reduction_indices")[0],
            "mean_output_shape": _out_shape([n for n in nodes if n["name"] == "huber_loss/Mean"][0]),
            "num_elements": _const(nodes, "huber_loss/weighted_loss/num_elements")[0],
            "final_division": [n["op"] for n in nodes if n["name"] == "huber_loss/weighted_loss/value"][0],
        }
        f["q_action"] = {
            "one_hot_shape": _out_shape([n for n in nodes if n["name"] == "one_hot"][0]),
            "mul_shape": _out_shape([n for n in nodes if n["name"] == "Mul"][0]),
            "sum_axis": _const(nodes, "Sum/reduction_indices")[0],
            "sum_shape": _out_shape([n for n in nodes if n["name"] == "Sum"][0]),
        }
    else:
        names = sorted({n["name"].split("/")[0] for n in nodes if "mean_squared_error" in n["name"]})
        f["loss"] = {"kind": "mse", "scopes": names,
                     "num_elements": [_const(nodes, n["name"])[0] for n in nodes
                                      if n["name"].endswith("weighted_loss/num_elements")]}
    bp = _fn(fns, "_batch_predict_max_future_reward_")
    f["batch_predict_max_future_reward"] = {"inputs": bp["inputs"][:1], "reduce": [n["op"] for n in bp["nodes"]
                                                                               if n["op"] in ("Max", "ArgMax")]}
    pa = _fn(fns, "_predict_action_")
    f["predict_action"] = {"inputs": pa["inputs"][:1], "reduce": [n["op"] for n in pa["nodes"] if n["op"] in ("Max", "ArgMax")]}
    return f


MODELS = {"breakout": "ql_model_breakout_84x84x4_3_32", "ballgame": "ql_model_ballgame_3x3x4_5_512"}


def main(ref="/root/reference"):
    here = os.path.dirname(os.path.abspath(__file__))
    for key, d in MODELS.items():
        rel = f"src/ql-with-tensorflow/python_model/saved/{d}"
        out = {"source": rel + "/{saved_model.pb,keras_metadata.pb}", "facts": facts(os.path.join(ref, rel))}
        with open(os.path.join(here, f"{key}_graph_facts.json"), "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
            fh.write("\n")
        print("wrote", key)


if __name__ == "__main__":
    main(*sys.argv[1:])
