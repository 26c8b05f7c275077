{{- define "llm-slo-agent.name" -}}llm-slo-agent{{- end -}}
{{- define "llm-slo-agent.labels" -}}
app.kubernetes.io/name: {{ include "llm-slo-agent.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
helm.sh/chart: {{ .Chart.Name }}-{{ .Chart.Version }}
{{- end -}}
{{- define "llm-slo-agent.selector" -}}
app.kubernetes.io/name: {{ include "llm-slo-agent.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}
