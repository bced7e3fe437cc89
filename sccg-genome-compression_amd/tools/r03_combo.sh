#!/bin/bash
set -o pipefail
bash sccg-genome-compression_amd/tools/r03_pipe.sh && bash sccg-genome-compression_amd/tools/r03_chain2.sh
