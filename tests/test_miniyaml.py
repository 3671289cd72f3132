"""The dependency-free kubeconfig YAML subset parser agrees with PyYAML or refuses."""
import pytest
import yaml
from hypothesis import given, settings, strategies as st

from k8s_gpu_node_checker_amd.utils import miniyaml

KUBECTL_STYLE = """apiVersion: v1
clusters:
- cluster:
    certificate-authority-data: LS0tLS1CRUdJTiBDRVJUSUZJQ0FURS0tLS0tCk1JSUM=
    server: https://10.0.0.1:6443   # the API
  name: prod
- cluster:
    insecure-skip-tls-verify: true
    server: "https://[fd00::1]:443"
  name: v6
contexts:
- context:
    cluster: prod
    namespace: default
    user: admin
  name: prod
current-context: prod
kind: Config
preferences: {}
users:
- name: admin
  user:
    exec:
      apiVersion: client.authentication.k8s.io/v1beta1
      args:
      - --region
      - us-west-2
      - eks
      - get-token
      command: aws
      env:
      - name: AWS_PROFILE
        value: 'it''s prod'
      interactiveMode: IfAvailable
      provideClusterInfo: false
- name: tok
  user:
    token: "abc\\tdef"
    username: null
    extra: ~
"""


def test_kubectl_style_matches_pyyaml():
    assert miniyaml.loads(KUBECTL_STYLE) == yaml.safe_load(KUBECTL_STYLE)


@pytest.mark.parametrize("text", ["a: &x 1\\nb: *x\n", "a: |\n  multi\n  line\n", "a: [1, 2]\n", "a: {b: 1}\n",
                                  "a: !!str 1\n", "---\na: 1\n---\nb: 2\n", "a: 1.5\n", "a: 0755\n",
                                  "a: b\n  c\n"])
def test_unsupported_constructs_are_refused(text):
    with pytest.raises(miniyaml.Unsupported):
        miniyaml.loads(text)


def test_empty_document():
    assert miniyaml.loads("") is None and miniyaml.loads("# only a comment\n") is None


words = st.text(alphabet=st.characters(whitelist_categories=("Ll", "Lu", "Nd"), whitelist_characters="-_./:"),
                min_size=1, max_size=12)
leaf = st.one_of(words, st.integers(-1000, 1000), st.booleans(), st.none())
tree = st.recursive(leaf, lambda ch: st.one_of(st.lists(ch, max_size=3), st.dictionaries(words, ch, max_size=3)),
                    max_leaves=12)


@settings(max_examples=300)
@given(st.dictionaries(words, tree, min_size=1, max_size=4), st.sampled_from([2, 4]))
def test_safe_dump_roundtrip(doc, indent):
    text = yaml.safe_dump(doc, default_flow_style=False, indent=indent)
    try:
        got = miniyaml.loads(text)
    except miniyaml.Unsupported:
        return
    assert got == yaml.safe_load(text)


# --- YAML 1.1 plain-scalar resolution, pinned against PyYAML on hand-written (not safe_dump'd) text ---

YAML11_FORMS = [
    # every bool spelling PyYAML's resolver knows, plus near misses
    "yes", "Yes", "YES", "no", "No", "NO", "true", "True", "TRUE", "false", "False", "FALSE",
    "on", "On", "ON", "off", "Off", "OFF", "yEs", "nO", "oN", "y", "n", "Y", "N", "tRUE", "yes please", "no-proxy",
    # null forms
    "~", "null", "Null", "NULL", "nULL", "~x", "null!",
    # int forms: decimal, octal, hex, binary, underscores, sexagesimal, signs
    "0", "7", "-0", "+5", "-12", "123", "007", "0755", "0o17", "0x1F", "0X1F", "-0x1f", "0b101", "+0b1", "1_000",
    "1:30", "190:20:30", "08", "09",
    # float forms
    "1.5", "-1.5", "1.", "1e3", "1.0e+3", "1.0e3", "6.8523015e+5", ".5", "-.5", ".inf", "-.Inf", "+.INF", ".NaN",
    ".nan", "1:30.5", "1_0.5", "1.2.3", "10.0.0.1", "1e", "0x", "+", "-", "++1", ".", "..", ".x",
    # timestamps
    "2001-12-14", "2001-12-14t21:59:43.10-05:00", "2001-12-14 21:59:43.10 -5", "2001-1-1",
    # merge / value / indicators
    "<<", "=", "==", "<", "-x", "--region", "?x", ":x", "x:", "a:b", "a #b", "a#b", "a: b", "x: ", "@x", "`x",
    "%x", "!x", "&x", "*x", "|", ">", "[x]", "{x}", ",x", "]x", "}x", "#x",
    # ordinary strings kubeconfigs hold
    "v1", "https://10.0.0.1:6443", "0.0.0.0/0", "client.authentication.k8s.io/v1beta1", "IfAvailable", "Config",
    "it's", 'say "hi"', "a  b", "a\tb", "\\x",
]


def _same(a, b):
    """Equality that also tells True from 1 and 1 from 1.0 (Python's == does not)."""
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return len(a) == len(b) and all(any(_same(k, k2) and _same(v, b[k2]) for k2 in b) for k, v in a.items())
    if isinstance(a, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    return a == b


def _quoted(s, q):
    if q == "'":
        return "'" + s.replace("'", "''") + "'"
    if q == '"':
        return '"' + s.replace("\\", "\\\\").replace('"', '\\"').replace("\t", "\\t") + '"'
    return s


def _docs(s):
    for q in ("", "'", '"'):
        v = _quoted(s, q)
        yield f"k: {v}\n"
        yield f"{v}: x\n"
        yield f"- {v}\n- {v}\n"
        yield f"a:\n  - {v}\n  - k: {v}\n    {v}: 1\nb: {v}   # trailing comment\n"
        yield f"{v}\n"


def _agrees(text):
    try:
        got = miniyaml.loads(text)
    except miniyaml.Unsupported:
        return True  # the caller falls back to PyYAML
    want = yaml.safe_load(text)  # raises if miniyaml accepted what PyYAML rejects -> test fails
    return _same(got, want)


@pytest.mark.parametrize("form", YAML11_FORMS)
def test_yaml11_plain_scalars_match_pyyaml_or_refuse(form):
    for text in _docs(form):
        assert _agrees(text), (form, text, miniyaml.loads(text), yaml.safe_load(text))


@pytest.mark.parametrize("form", ["yes", "no", "on", "off", "true", "false", "TRUE", "Off", "y", "n", "~", "null", "0"])
def test_yaml11_keys_and_values_resolved_not_left_as_strings(form):
    """The round-2 bug: ``no`` came back as the string 'no' (truthy) instead of False."""
    got = miniyaml.loads(f"k: {form}\n{form}: v\n")
    want = yaml.safe_load(f"k: {form}\n{form}: v\n")
    assert _same(got, want)


scalar_text = st.text(alphabet=st.sampled_from(list("yesnotrufalYESNOTRUFAL~0123456789.+-_:xX#@!&*'\"%` \t<=eEiInNfF")),
                      min_size=1, max_size=8)


@settings(max_examples=1500, deadline=None)
@given(scalar_text, st.booleans())
def test_handwritten_scalars_differential(s, q):
    for text in _docs(s if q else s.strip() or "x"):
        assert _agrees(text), text


def test_insecure_skip_tls_verify_no_keeps_verification(tmp_path):
    from k8s_gpu_node_checker_amd.kube import config as kc
    for word, insecure in (("no", False), ("off", False), ("No", False), ("OFF", False), ("false", False),
                           ("yes", True), ("on", True), ("true", True)):
        p = tmp_path / f"kc-{word}"
        p.write_text(f"""apiVersion: v1
clusters:
- cluster:
    insecure-skip-tls-verify: {word}
    server: https://10.0.0.1:6443
  name: c
contexts:
- context:
    cluster: c
    user: u
  name: x
current-context: x
users:
- name: u
  user:
    token: abc
""")
        conn = kc.load_kube_config(str(p))
        assert conn.insecure is insecure, word


@pytest.mark.parametrize("val", ["'no'", '"false"', "0", "1", "[]", "nope"])
def test_insecure_skip_tls_verify_must_be_a_boolean(tmp_path, val):
    from k8s_gpu_node_checker_amd.kube import config as kc
    from k8s_gpu_node_checker_amd.kube.errors import ConfigException
    p = tmp_path / "kc"
    p.write_text(f"""clusters:
- cluster:
    insecure-skip-tls-verify: {val}
    server: https://10.0.0.1:6443
  name: c
contexts:
- context: {{cluster: c}}
  name: x
current-context: x
""")
    with pytest.raises(ConfigException, match="insecure-skip-tls-verify"):
        kc.load_kube_config(str(p))


_struct_piece = st.text(alphabet=st.sampled_from(list("yesnotrufalYESNO~0123456789.+-_:x#@!&*'\"% <=eEnN[]{},?|>\\/")),
                        max_size=8)
_struct_line = st.tuples(st.sampled_from([0, 1, 2, 4]), st.sampled_from(["", "- ", "- - "]), _struct_piece,
                         st.sampled_from([": ", ":", "", " # c"]), _struct_piece)


@settings(max_examples=800, deadline=None)
@given(st.lists(_struct_line, min_size=1, max_size=5))
def test_handwritten_structures_differential(lines):
    """Hand-written block structure (indent, sequences, keys, comments) around hand-written scalars."""
    text = "".join(" " * i + d + a + sep + b + "\n" for i, d, a, sep, b in lines)
    assert _agrees(text), text


@pytest.mark.parametrize("text", [KUBECTL_STYLE.replace("\n", "\r\n"), "a: b\r\nc: d\r", "a: 'x\ry'\n", "a: b\rc: d\n"])
def test_line_endings_match_pyyaml_or_refuse(text):
    assert _agrees(text)
