set -e
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/c2_sequence.py 1000 16 > gpurun_out/r06_c2_sequence.json 2> gpurun_out/r06_c2_sequence.err
timeout -k 10 500 python -u tools/c5_pipeline.py > gpurun_out/r06_c5_pipeline.json 2> gpurun_out/r06_c5_pipeline.err
