"""Medical-device training assistant (multi-turn RAG over instructions-for-use manuals)."""
from generativeaiexamples_amd.examples.medical_device import MedicalDeviceAssistant  # noqa: F401
