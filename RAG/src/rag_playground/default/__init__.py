"""Reference-path shim: the playground lives in generativeaiexamples_amd.playground."""
from generativeaiexamples_amd.playground import ChatClient, create_app  # noqa: F401
