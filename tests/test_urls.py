"""utils/urls.py agrees with urllib.parse (urlsplit / quote(safe=""))."""
from urllib.parse import quote, urlsplit

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from k8s_gpu_node_checker_amd.utils import urls

CASES = ["https://10.0.0.1:6443", "http://127.0.0.1:8080/base/path?x=1", "https://API.Example.com",
         "https://[::1]:6443/", "https://[FE80::1]", "http://host:/p", "http://:80/", "https://h.example.com:443",
         "HTTP://Host", "https://u:p@h:1/", "https://h/%20", "http://h#frag", "https://hooks.slack.com/services/T/B/X",
         "https://h:99999", "https://h:x", "http://h\t/", "http://é.example/", "noscheme", "/path/only", "",
         "ftp://h/x", "http://[::1", "a://]", "http://h]:1/", "https://h:1:2", "http://h?q", "http://h:65535"]


def _ref(u):
    p = urlsplit(u)
    return (p.scheme, p.netloc, p.hostname, p.port, p.path, p.query)


def _ours(u):
    return urls.split(u).astuple()


@pytest.mark.parametrize("u", CASES)
def test_split_matches_urlsplit(u):
    try:
        ref = _ref(u)
    except ValueError as e:
        with pytest.raises(ValueError):
            _ours(u)
        return
    assert _ours(u) == ref


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet="htps:/[]1:.aBZ%@?#x-_ 90", max_size=30))
def test_split_fuzz(u):
    try:
        ref = _ref(u)
    except ValueError:
        with pytest.raises(ValueError):
            _ours(u)
        return
    assert _ours(u) == ref


@settings(max_examples=300, deadline=None)
@given(st.text(max_size=20))
def test_quote_matches(s):
    assert urls.quote(s) == quote(s, safe="")
