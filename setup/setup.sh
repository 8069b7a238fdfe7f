#!/usr/bin/env bash
# Build and start the service container (reference setup/setup.sh:1-20).
# Fixes vs the reference: works from any cwd, and the volume check looks at the exit status
# (docker prints "No such volume" on stderr, so the reference's stdout grep never matched).
set -euo pipefail
cd "$(dirname "$0")/.."

echo "Checking Image Storage Volume..."
if ! docker volume inspect photoanalysisserver_images >/dev/null 2>&1; then
  echo "Creating Image Storage Volume..."
  docker volume create --name=photoanalysisserver_images
else
  echo "Image Storage Volume Already Exists!"
fi

echo "Building Docker Container"
docker-compose build

echo "Starting Docker Container..."
docker-compose up -d
