"""Test stand-in for python-dotenv: ``load_dotenv`` is a no-op (tests pass env explicitly)."""


def load_dotenv(*args, **kwargs):
    return False
