{{- define "ome-amd.name" -}}{{ .Release.Name }}-ome-amd{{- end -}}
{{- define "ome-amd.labels" -}}
app.kubernetes.io/name: ome-amd-manager
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}
