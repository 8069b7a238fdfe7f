# MI355X (gfx950) serving image.  Reference: tiangolo/uvicorn-gunicorn-fastapi:python3.7 +
# `pip install -r requirements.txt` (reference Dockerfile:1-7).  Here the base is a ROCm
# PyTorch image; the HIP kernels are compiled for gfx950 at build time (hipcc ships in it).
ARG BASE_IMAGE=rocm/pytorch:latest
FROM ${BASE_IMAGE}

WORKDIR /app
COPY . /app

RUN pip --no-cache-dir install -r requirements.txt \
 && python -m mlmicroservicetemplate_amd build

# dmabuf IPC (RCCL / cross-process tensor sharing) on current amdgpu drivers
ENV HSA_ENABLE_IPC_MODE_LEGACY=0
EXPOSE 5005
CMD ["python", "-m", "mlmicroservicetemplate_amd", "serve", "--env-file", "/app/.env"]
