for c in C2 C3 C4; do
  s=2; timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['counters']; s=c['segments']
print('$c', d['value'], 'seg/sample %.3f'%(s/c['samples']), 'nodes/seg %.2f'%(c['node_visits']/s), 'node simd eff %.3f'%(c['node_visits']/64/max(1,c['wave_node_iters'])), 'leaf eff %.3f'%((c['sphere_tests']+c['quad_tests'])/64/max(1,c['wave_leaf_iters'])), 'trip eff %.3f'%(s/64/c['wave_trips']), 'shade eff %.3f'%(c['shade_events']/64/max(1,c['wave_shade_iters'])), 'wnode/trip %.2f'%(c['wave_node_iters']/c['wave_trips']), 'wleaf/trip %.2f'%(c['wave_leaf_iters']/c['wave_trips']), 'wshade/trip %.2f'%(c['wave_shade_iters']/c['wave_trips']))"
done
