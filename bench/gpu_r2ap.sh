# combined: route probe + training batch sweep (r2an), one-shot fused stage+signal validation (r2ao)
bash bench/gpu_r2an.sh && bash bench/gpu_r2ao.sh
