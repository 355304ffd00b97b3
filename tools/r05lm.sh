#!/bin/bash
bash tools/r05l.sh || exit $?
bash tools/r05m.sh
