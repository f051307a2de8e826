"""yalm_amd — MI355X-native (gfx950) single-batch decode engine with the
reference yalm's Model/InferenceState API.

The compute path is the HIP shared library ``libyalm_hip.so`` (C ABI in
``include/yalm_hip.h``), bound by ``yalm_amd.runtime``. There is no CPU
fallback: importing ``yalm_amd.runtime`` without the built library raises.

Pure-Python helpers that need no device: ``yalm_amd.yalmfile`` (.yalm
reader/writer), ``yalm_amd.convert`` (HF -> .yalm), ``yalm_amd.tokenizer``.
"""
