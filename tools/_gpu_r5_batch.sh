S='bash tools/gpu_steps.sh'
$S "420|native|python -u -m pytest tests/test_native_engine.py -m gpu -x -v --timeout 360 --timeout-method thread"
