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
