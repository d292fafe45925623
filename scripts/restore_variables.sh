#!/usr/bin/env bash
# Restore a saved session: `source scripts/restore_variables.sh [variables.sh]`
FILE="${1:-variables.sh}"
if [ ! -f "$FILE" ]; then echo "$FILE not found" >&2; return 1 2>/dev/null || exit 1; fi
# shellcheck disable=SC1090
. "$FILE"
echo "restored variables from $FILE"
