bash scripts/ab_libs.sh r2aa "c4 c3" base xin
