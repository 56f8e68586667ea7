# round-4: pingpong8om with spread boundary stores (pingpong8omd) on ragged multi-round shapes
PYARGS="--variants pingpong8omd --repeats 30" bash tools/gpu_run.sh r4_omd_race py:tools/race_screen.py && \
PYARGS="--sizes 6904x5392x6352,6520x5440x5520,5504x8056x5440,6568x7272x4512,6480x6984x3552,4752x8176x7288,6000x7000x3000,3000x9000x4096,5000x4104x4096,7784x6472x1464,5184x4120x3184,4808x4424x2824 --variants default,pingpong8cm,pingpong8om,pingpong8omd --rounds 7 --iters 20" bash tools/gpu_run.sh r4_omd_time py:tools/gemm_check.py
