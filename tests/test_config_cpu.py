"""CPU tests of ConfigParser (src/ConfigParserYAML.cpp:10-118): the reference reads its
config with YAML::LoadFile, so the same document must parse identically as the shipped
JSON (YAML flow style) and as block YAML; no GPU is involved."""
import json
import os

import pytest

from conftest import CONFIG

otp = pytest.importorskip("online_traj_planner")


def _yaml_scalar(v, style):
    if isinstance(v, bool):
        return {"plain": "true" if v else "false", "yes": "yes" if v else "no", "quoted": "True" if v else "False"}[style]
    if isinstance(v, (int, float)):
        return repr(v)
    if style == "quoted":
        return json.dumps(v)
    if style == "yes":
        return "'" + v.replace("'", "''") + "'"
    return v


def _to_yaml(d, style, indent=0):
    """Block YAML of a JSON document: mappings by indentation, number lists as flow
    sequences (one spread over two lines), comments sprinkled in."""
    pad = " " * indent
    out = []
    for k, v in d.items():
        key = json.dumps(k) if style == "quoted" else str(k)
        if isinstance(v, dict):
            out.append(f"{pad}{key}:   # {k}")
            out.extend(_to_yaml(v, style, indent + 2))
        elif isinstance(v, list):
            items = [_yaml_scalar(x, style) for x in v]
            if style == "yes":  # block sequence
                out.append(f"{pad}{key}:")
                out.extend(f"{pad}- {x}" for x in items)
            elif len(items) == 3:
                out.append(f"{pad}{key}: [{items[0]}, {items[1]},")
                out.append(f"{pad}    {items[2]}]")
            else:
                out.append(f"{pad}{key}: [{', '.join(items)}]")
        else:
            out.append(f"{pad}{key}: {_yaml_scalar(v, style)}")
    return out


@pytest.fixture(scope="module")
def ref_dict():
    return otp.load_config(CONFIG)


def test_json_config_values(ref_dict):
    d = json.load(open(CONFIG))
    assert ref_dict["path_planner"]["samples_fmt"] == d["path_planner_properties"]["samples_fmt"]
    assert ref_dict["path_planner"]["planner"] == d["path_planner_properties"]["planner"]
    assert ref_dict["world"]["inflate_radius"]["gate"] == d["world_properties"]["inflate_radius"]["gate"]
    sizes = [tuple(s / 2 for s in o["size"]) for o in d["component_geometry"]["large_portal"].values()]
    assert [o["half_size"] for o in ref_dict["gate_geometry"][0]] == sizes


@pytest.mark.parametrize("style", ["plain", "yes", "quoted"])
def test_block_yaml_equals_json(tmp_path, ref_dict, style):
    d = json.load(open(CONFIG))
    text = "# drone racing config\n---\n" + "\n".join(_to_yaml(d, style)) + "\n"
    p = tmp_path / "config.yaml"
    p.write_text(text)
    assert otp.load_config(str(p)) == ref_dict


def test_flow_yaml_with_plain_keys(tmp_path, ref_dict):
    # a one-document flow mapping that is not strict JSON (unquoted keys)
    d = json.load(open(CONFIG))
    body = json.dumps(d).replace('"path_planner_properties"', "path_planner_properties")
    p = tmp_path / "config.yaml"
    p.write_text(body)
    assert otp.load_config(str(p)) == ref_dict


@pytest.mark.parametrize("bad,msg", [
    ("a: 1\n  b: 2\n", "YAML"),
    ("a: &x 1\n", "anchors"),
    ("a: |\n  text\n", "block scalars"),
])
def test_yaml_errors(tmp_path, bad, msg):
    p = tmp_path / "bad.yaml"
    p.write_text(bad)
    with pytest.raises(RuntimeError, match=msg):
        otp.load_config(str(p))


def test_missing_key_and_file(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("component_geometry:\n  obstacle: {}\n")
    with pytest.raises(RuntimeError, match="missing key"):
        otp.load_config(str(p))
    with pytest.raises(RuntimeError, match="bad file"):
        otp.load_config(os.path.join(str(tmp_path), "nope.yaml"))


def test_yaml_plain_scalars_keep_their_text(tmp_path, ref_dict):
    """Plain scalars that YAML would type as bool (on, y, no ...) or that strtod alone
    would read as a number (nan, inf, 0x10) stay readable as strings, as yaml-cpp's
    .as<std::string>() returns their text: here a component called "on" (a gate type's
    name, src/ConfigParserYAML.cpp:21-52) and OBB names "nan" / "0x10"."""
    d = json.load(open(CONFIG))
    mapping = d["gate_id_to_name_mapping"]
    old = mapping["1"]
    mapping["1"] = "on"
    d["component_geometry"]["on"] = d["component_geometry"].pop(old)
    d["component_properties"]["on"] = d["component_properties"].pop(old)
    obbs = list(d["component_geometry"]["on"].values())
    obbs[0]["name"], obbs[1]["name"] = "nan", "0x10"
    text = "\n".join(_to_yaml(d, "plain")) + "\n"
    assert "\n  1: on" in text or "1: on" in text
    p = tmp_path / "config.yaml"
    p.write_text(text)
    got = otp.load_config(str(p))
    assert [o["name"] for o in got["gate_geometry"][1][:2]] == ["nan", "0x10"]
    strip = lambda g: {t: [{k: v for k, v in o.items() if k != "name"} for o in obbs] for t, obbs in g.items()}  # noqa: E731
    assert strip(got["gate_geometry"]) == strip(ref_dict["gate_geometry"])
    assert got["path_planner"] == ref_dict["path_planner"]
