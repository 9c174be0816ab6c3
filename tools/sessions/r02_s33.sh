set -u
bash tools/sweep_resumable.sh 14 60 r02_sweep_medium_s16o14_v11 && bash tools/sweep_resumable.sh 1 130 r02_sweep_medium_s16o1_v12 && bash tools/sweep_resumable.sh 3 180 r02_sweep_medium_s16o3_v12
