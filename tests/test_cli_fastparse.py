"""cli._fast_parse (the argparse-free parse of a plain command line) must agree with argparse exactly,
and hand everything else to argparse (help, usage errors, abbreviations)."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from k8s_gpu_node_checker_amd import cli

VALUES = {"--slack-retry-count": ["0", "5", "x", "-1", "3.5"], "--kube-timeout": ["0.5", "30", "abc", "1e3"],
          "--gpu-source": ["capacity", "allocatable", "bogus"], "--health-policy": ["off", "require", "x"],
          "--kubeconfig": ["/tmp/kc", "", "-"], "--xgmi-links": ["0", "8", "seven"]}


def _argparse(argv):
    try:
        return vars(cli.build_parser().parse_args(argv))
    except SystemExit as e:
        return ("exit", e.code)


def _token_lists():
    flags = [f for _, f, _ in cli._FLAGS if f != "--help-all"]

    def one(flag):
        opts = dict((f, o) for _, f, o in cli._FLAGS)[flag]
        if opts.get("action") == "store_true":
            return st.sampled_from([[flag], [flag + "=1"]])
        vals = VALUES.get(flag, ["v", "12", "a b"])
        return st.sampled_from(vals).flatmap(lambda v: st.sampled_from([[flag, v], [flag + "=" + v], [flag]]))
    extra = st.sampled_from([["--jso"], ["-h"], ["pos"], ["--unknown"], ["--json", "--json"]])
    return st.lists(st.one_of(st.sampled_from(flags).flatmap(one), extra), max_size=6).map(
        lambda xs: [t for x in xs for t in x])


@settings(max_examples=400, deadline=None)
@given(_token_lists())
def test_fast_parse_agrees_with_argparse(argv):
    fast = cli._fast_parse(argv)
    ref = _argparse(argv)
    if fast is None:
        return  # argparse handles it (possibly an error / help)
    assert not isinstance(ref, tuple), (argv, ref)
    assert vars(fast) == ref, argv


def test_plain_command_lines_take_the_fast_path():
    for argv in ([], ["--json"], ["--kubeconfig", "/k", "--json"], ["--kubeconfig=/k", "--mi355x"],
                 ["--slack-webhook", "http://x", "--slack-only-on-error", "--slack-retry-count", "0"]):
        assert cli._fast_parse(argv) is not None, argv
        assert vars(cli._fast_parse(argv)) == _argparse(argv)
    for argv in (["--help"], ["-h"], ["--jso"], ["--slack-retry-count", "x"], ["--gpu-source", "bogus"],
                 ["--kubeconfig"], ["pos"], ["--json=1"]):
        assert cli._fast_parse(argv) is None, argv


def test_cli_does_not_import_argparse_for_a_plain_check(run_cli, mock_cluster, tmp_path):
    import subprocess
    import sys
    from k8s_gpu_node_checker_amd.testing import fixtures
    srv = mock_cluster([fixtures.realistic_node("a")])
    kc = str(tmp_path / "kc")
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    write_kubeconfig(kc, srv.url)
    code = ("import sys, runpy; sys.argv = ['check-gpu-node', '--kubeconfig', %r, '--json']\n"
            "try:\n    runpy.run_path(%r, run_name='__main__')\nexcept SystemExit as e:\n    rc = e.code\n"
            "print('MODS', 'argparse' in sys.modules, 'socket' in sys.modules, 'ctypes' in sys.modules, rc)"
            % (kc, cli.__file__.replace("k8s_gpu_node_checker_amd/cli.py", "check-gpu-node.py")))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    line = [x for x in p.stdout.splitlines() if x.startswith("MODS")][0]
    assert line == "MODS False False False 0", (line, p.stderr[-2000:])


@pytest.mark.parametrize("argv", [["--slack-retry-count", "x"], ["--gpu-source", "bogus"]])
def test_usage_errors_still_exit_2(run_cli, argv):
    p = run_cli(argv)
    assert p.returncode == 2 and "error:" in p.stderr
